/*
 * mdqt.h — C ABI of the MI355X-native MDQT engine (libmdqt.so).
 *
 * Drop-in boundary for the hot path of the reference program
 *   laserCoolingPlusExpansionMDQTSpeedUp.cpp        ("SpeedUp" below, tlangin/MDQTPlasmaSims)
 * The reference has no plugin API: its seam is a set of void functions over globals
 * (SpeedUp:176-185 prototypes) plus the process interface `exe <job>` (SpeedUp:1145).
 * Every entry point below names the reference function it replaces (file:line).
 *
 * Conventions
 *   - opaque context, int status (0 = ok, <0 = error; mdqt_last_error() has the message);
 *   - host buffers are caller-owned; R/V/F are SoA [3][ld] row-major exactly like the
 *     reference's `double R[3][N0+1000]` (SpeedUp:126-129) with the row stride `ld` explicit;
 *   - psi is [N][12][2] interleaved (re, im): the storage order of `cx_mat wvFns[N]`
 *     (12x1 column, SpeedUp:151);
 *   - device state stays resident in HBM between calls; get/set are the only host syncs;
 *   - one context is not reentrant; distinct contexts are independent (thread-safe).
 * No torch types, no HIP types: the stream is passed as void* (a hipStream_t).
 */
#ifndef MDQT_H
#define MDQT_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define MDQT_NUM_STATES 12   /* numStates, SpeedUp:153 */
#define MDQT_NBINS 2001      /* velocity-distribution bins, SpeedUp:120-123, :340-344 */

/* User inputs of the reference (compile-time globals / #defines at SpeedUp:56-85), same
 * names, same defaults (mdqt_default_params), plus the engine's own extensions. */
typedef struct mdqt_params {
    double Ge;            /* SpeedUp:60  Gamma_e; kappa = sqrt(3 Ge), lDeb = 1/kappa (:295)   */
    double tmax;          /* SpeedUp:63  end time (omega_E^-1)                                */
    double density;       /* SpeedUp:65  1e14 m^-3                                            */
    double sig0;          /* SpeedUp:66  initial plasma size (mm)                             */
    double Te;            /* SpeedUp:67  electron temperature (K)                             */
    double fracOfSig;     /* SpeedUp:68  position in the expanding cloud (0 = no expansion)   */
    double detuning;      /* SpeedUp:70  S-P detuning (units of gamma)                        */
    double detuningDP;    /* SpeedUp:71  D-P detuning                                         */
    double Om;            /* SpeedUp:72  S-P Rabi frequency                                   */
    double OmDP;          /* SpeedUp:73  D-P Rabi frequency                                   */
    int N0;               /* SpeedUp:69  nominal ion number                                   */
    int newRun;           /* SpeedUp:61  1 = init(), 0 = readConditions(c0)                   */
    int c0;               /* SpeedUp:62  MD-step index to resume from                          */
    int sampleFreq;       /* SpeedUp:78  output every sampleFreq MD steps                     */
    int reNormalizewvFns; /* SpeedUp:74                                                       */
    /* ---- extensions ---- */
    int qt_enabled;       /* 1 = MDQT (reference); 0 = MD-only (qstep body skipped, t advances) */
    int rng_mode;         /* 1 = Philox4x32-10 keyed (seed, job) x (global ion, qstep): fast,
                           *     reproducible, the same draws for an ion at any world size
                           *     (default; trajectories are bit-identical across world sizes
                           *     with the owner-computes rows scheme, N <= 65,536, and agree to
                           *     rounding with the Newton-3 block scheme above that — its rank
                           *     partials are summed in the reduce-scatter's order);
                           * 0 = the reference's own drand48 stream in its consumption order
                           *     (SpeedUp:486, :575-687; one stream, world_size 1): trajectory
                           *     parity with the 1-thread reference, one launch per substep   */
    uint32_t seed;        /* srand48 seed for init (reference: time(NULL)+job, SpeedUp:1219)   */
    uint32_t job;         /* SpeedUp:1145 argv[1]                                               */
    int device;           /* HIP device ordinal (-1 = current device)                           */
    int world_size;       /* ions sharded over world_size contexts (1 = whole system here)     */
    int rank;             /* this context's slab: ions [rank*S, min((rank+1)*S, N))             */
    int force_segments;   /* j-split of the force sum (0 = auto, a function of N only)         */
    int qt_model;         /* level scheme of qstep(): 0 = SpeedUp Sr+ 12-level laser cooling (default);
                           * optical pumping ("spin tagging", Philox stream and qt_math 2 only):
                           * 1 = 408 nm linear, 7 levels (randomFrozenStartTag408Linear.cpp:396,
                           *     MonteCarloFollowedByQTTagging408Linear.cpp:555),
                           * 2 = 408 nm quad, 7 levels (randomFrozenStartTag408Quad.cpp:399),
                           * 3 = 422 nm linear, 5 levels (randomFrozenStartTag422Linear.cpp:390).
                           * Pumping models use states 0..6 / 0..4 of the 12-state psi layout. */
    char saveDirectory[256]; /* SpeedUp:56 */
    /* ---- the optical-pumping programs' main() (mdqt_run_pump; qt_model 1-3) ---- */
    double tpumpreal;     /* randomFrozenStartTag408Linear.cpp:58  pump duration (s)           */
    double tstartV0;      /* :78  pump window start (omega_E^-1); window = (tstartV0, tendV0)   */
} mdqt_params;

typedef struct mdqt_ctx mdqt_ctx;

/* ---- lifecycle ---- */
void        mdqt_default_params(mdqt_params* p);            /* SpeedUp:56-85 defaults          */
/* the pumping programs' defaults: model 1 = randomFrozenStartTag408Linear.cpp:52-80,
 * 2 = randomFrozenStartTag408Quad.cpp:55-81, 3 = randomFrozenStartTag422Linear.cpp:52-78 */
void        mdqt_default_params_pump(mdqt_params* p, int qt_model);
int         mdqt_create(const mdqt_params* p, mdqt_ctx** out); /* + constant operators :1163-1215 */
void        mdqt_destroy(mdqt_ctx* c);
const char* mdqt_last_error(void);                           /* thread-local message            */
int         mdqt_device_count(void);                         /* HIP devices visible             */
const char* mdqt_version(void);

/* ---- derived constants (SpeedUp:79-85, :146-149, :295-297, :1181-1215) ----
 * plus the engine's state: "force_scheme", "force_slots", "force_sort", "force_skip_radius",
 * "force_tail_bound", "force_far_radius", "force_far_bound" (see the tuning knobs), "qt_kernel" /
 * "qt_kernel_nseg" (the substep kernel instance of the last launch and the force partials it
 * summed; codes of mdqt_internal.hpp QTKernel: 1 = the C2 production instance), "md_step_fused";
 * NaN for an unknown name */
double      mdqt_get_const(const mdqt_ctx* c, const char* name);

/* ---- state ---- */
int         mdqt_init(mdqt_ctx* c);                          /* init(), SpeedUp:289-348         */
int         mdqt_get_N(const mdqt_ctx* c);
double      mdqt_get_time(const mdqt_ctx* c);
int         mdqt_set_time(mdqt_ctx* c, double t);
uint64_t    mdqt_get_qstep_index(const mdqt_ctx* c);
int         mdqt_set_qstep_index(mdqt_ctx* c, uint64_t q);
/* rng_mode 0: the 48-bit drand48 state X after the draws consumed so far (glibc layout) */
int         mdqt_get_drand48_state(mdqt_ctx* c, uint64_t* x);
int         mdqt_get_counters(const mdqt_ctx* c, int* c0, unsigned* counter, double* Epot, double* Epot0);
/* Whole-system state (all N ions; with world_size > 1 only this rank's slab of V/F/psi/tPart
 * is meaningful, R is the full gathered array). NULL pointers are skipped. */
int         mdqt_set_state(mdqt_ctx* c, int N, const double* R, const double* V, size_t ld,
                           const double* psi, const double* tPart, double t);
int         mdqt_get_state(mdqt_ctx* c, double* R, double* V, double* F, size_t ld,
                           double* psi, double* tPart, double* t);
int         mdqt_set_forces(mdqt_ctx* c, const double* F, size_t ld);

/* ---- hot path ---- */
int         mdqt_forces(mdqt_ctx* c);                        /* forces(),  SpeedUp:192-236      */
int         mdqt_step(mdqt_ctx* c);                          /* step(),    SpeedUp:418-430      */
int         mdqt_qstep(mdqt_ctx* c);                         /* qstep(),   SpeedUp:438-717      */
int         mdqt_substeps(mdqt_ctx* c, int n);               /* n x (step(); qstep()), F frozen;
                                                                 the body of SpeedUp:1376-1377,
                                                                 fused in one launch            */
int         mdqt_md_steps(mdqt_ctx* c, int n);               /* n x (forces(); c0++;
                                                                 ratio x (step(); qstep()))     */

/* Stateless kernel-level entry points on caller host arrays (explicit box and screening
 * length), for callers whose force law is the same Yukawa pair sum but whose box is not
 * SpeedUp's — e.g. MonteCarloFollowedByMDAndTempAnisotropy.cpp calculateAccelerations
 * (:387-448, acceleration = force at unit mass) and calculatePotentialEnergyForParticles
 * (:207-244).  R, F are [3][ld]; nseg = j-split (0 = auto); U[i] = sum_{j != i} u(r_ij);
 * variant 0 = the reference's exact operations, 1 = fast reciprocal form (<= 1e-13 rel). */
int         mdqt_forces_raw(int N, double L, double lDeb, const double* R, size_t ld, double* F,
                            int nseg, int device, int variant);
int         mdqt_potentials_raw(int N, double L, double lDeb, const double* R, size_t ld, double* U,
                                int nseg, int device, int variant);

/* ---- diagnostics / output ---- */
/* Work census of the Newton-3 block force kernel (N > 65,536, spatial order; this rank's block
 * pairs) for the current positions — the tile pairs of forces() by the path they take: out[0..15)
 * lane-steps (64 per step of a wave: 16 steps per evaluated sub-tile group, 4,096 per skipped tile
 * pair, 2,560 on a diagonal tile), out[15..30) distinct ion pairs; classes 0 skipped beyond L/2,
 * 1 skipped by the tail radius, 2 ragged last tile, 3 exact per-pair image, 4 exact uniform image,
 * 5 far per-pair, 6 far uniform, 7 very far per-pair, 8 very far uniform, 9 ultra far (f64)
 * uniform, 10 ultra far in f32, 11 skipped sub-tile groups of evaluated tile pairs, 12 mid
 * per-pair, 13 mid uniform, 14 ultra far (f64) with a one-axis per-pair image (round 6).  n >= 30.  Not
 * part of the reference's seam: the benchmark's roofline bookkeeping (VALU per evaluated pair). */
int         mdqt_force_census(mdqt_ctx* c, double* out, int n);
int         mdqt_epotential(mdqt_ctx* c, double* Epot);      /* Epotential(), SpeedUp:244-281   */
/* the per-ion pair-potential row sums U_i that Epotential() adds up (Epot = sum U_i / 2N), by ion index,
 * world 1 — the same device path as mdqt_epotential (tests of its error-bounded block forms) */
int         mdqt_potential_rows(mdqt_ctx* c, double* U, int n);
/* observables of output(), SpeedUp:917-1032: out7 = t, EkinX, EkinY, EkinZ, Epot,
 * Etot-Epot0, <vx>; Pvel [3][2001] (may be NULL); pops [N][3] = S,P,D (may be NULL). */
int         mdqt_observables(mdqt_ctx* c, double out7[7], double* Pvel, double* pops);
int         mdqt_setup_directories(mdqt_ctx* c);             /* SpeedUp:1145-1160               */
const char* mdqt_save_directory(const mdqt_ctx* c);
int         mdqt_output(mdqt_ctx* c);                        /* output(),  SpeedUp:917-1032     */
int         mdqt_write_conditions(mdqt_ctx* c, int c0);      /* writeConditions, :725-784       */
int         mdqt_read_conditions(mdqt_ctx* c, int c0);       /* readConditions,  :785-916       */
int         mdqt_run(mdqt_ctx* c);                           /* main() time loop, :1139-1383    */
/* Output files are formatted ("%lg", byte-identical to fprintf) and written by background threads
 * of the context.  mdqt_output / mdqt_write_conditions / mdqt_run return after their files are on
 * disk (inside mdqt_run the per-output files are written while the loop goes on, joined at the
 * end); mdqt_flush_files waits for any still in flight and reports the first I/O error. */
int         mdqt_flush_files(mdqt_ctx* c);
/* optical-pumping models: tag every ion spin-up with probability |<up|psi>|^2 —
 * measureSpinUps (randomFrozenStartTag408Linear.cpp:600, randomFrozenStartTag422Linear.cpp:568)
 * = tagParticles (MonteCarloFollowedByQTTagging408Linear.cpp:1022).  tags: [N] (may be NULL;
 * a sharded context fills its slab), *n_up: number tagged (this context's ions). */
int         mdqt_tag_spin_up(mdqt_ctx* c, int* tags, int* n_up);
/* The optical-pumping programs' main() (randomFrozenStartTag408Linear.cpp:981-1076, 408Quad :990-1086,
 * 422Linear :946-1031; qt_model 1-3): directory PumpTime..PumpStart..Det..Om..Density..Ge..NumIons..
 * (:990), init() or readConditions(c0); the time loop — leapfrog MD step (step() :377-394,
 * forces at the half-drifted positions) every plasmaToQuantumTimestepRatio quantum steps, qstep()
 * only inside the pump window (tstartV0, tstartV0 + tpumpreal 813490 sqrt(density)), t += dtQ
 * otherwise; at the first t >= tendV0 measureSpinUps() (:600, spinUpIons_timestep%06d.dat), output()
 * and the VAF; then output() every sampleFreq MD steps: energies.dat, taggedMoments.dat,
 * vel_distX_timestep%06d.dat of the spin-up ions (4001 bins, :799-935), VAF.dat (:938-975);
 * writeConditions(c0) at the end: ions_, spinUpIonsList_, conditions_ (:667-707).  Quantum jumps
 * and the tags draw from the Philox stream (the reference's shared drand48 is racy).
 * world_size 1. */
int         mdqt_run_pump(mdqt_ctx* c);
/* the spin-up list of the pumping run (N ints; 0 before measureSpinUps) */
int         mdqt_get_spin_up_list(mdqt_ctx* c, int* tags, int* n_up);

/* ---- tuning knobs ----
 *   "substep_kernel": 0 = auto, 1 = thread per ion, 2 = 16-lane group per ion
 *   "force_kernel":   1 = fast reciprocal form (default), 0 = the reference's exact operations
 *                     (the two differ by a few ulp per pair; both meet the 1e-13 force gate)
 *   "force_scheme":   0 = auto, 1 = owner-computes rows, 2 = Newton-3 tile pairs (one GPU),
 *                     3 = Newton-3 block pairs (auto above 65,536 ions; sharded: reduce-scatter)
 *   "force_sort":     block pairs only: 1 = Hilbert-curve order with skipping of tile pairs whose
 *                     boxes are >= the skip radius apart (default), 2 = the same order, nothing
 *                     skipped (bit-identical to 1 where the skip radius is L/2 — every BASELINE size
 *                     but N ~ 1e6, where 1 also skips the error-bounded tail), 0 = storage order
 *   "force_ax1":      block pairs in spatial order: 1 (default) = a tile pair whose minimum image
 *                     varies on one axis only takes the image per pair on that axis alone (the
 *                     other two shifted once per tile pair, as a uniform-image tile pair) — a
 *                     kernel instance of its own, launched where the skip radius reaches within
 *                     two tile widths of L/2 (C3, C5); 0 = the per-pair image on all three axes.
 *                     Forces agree to rounding (1e-13 of max |F|)
 *   "force_reduce_mask": block pairs in spatial order: 1 (default) = the slot reduction reads only the
 *                     j-slots the block kernel wrote (per-J-tile masks of the block distances whose J
 *                     step has work, from the plan), 0 = every j-slot (empty J steps write -0).  Bit
 *                     for bit the same forces (acc + -0 = acc)
 *   "force_tile_split": Newton-3 tiles: 1 (default) = the whole tile pairs of the kernel's last round of
 *                     workgroups (after the diagonal ones) run as two half workgroups each, their second
 *                     halves' rows in one extra slot (C2 on 256 CUs: 4 of 1,596; "force_tile_split_pairs"
 *                     reports the count, "device_cus" the device's compute units); 0 = whole tile pairs
 *                     only.  Forces agree to rounding (another summation order on the split tiles); the
 *                     options overlap / fused_step take the plain table.  The table follows the device's
 *                     CU count, so F's last bits (and trajectories) can differ between devices with
 *                     different counts: "force_split_cus" = n cuts it for n CUs on any device (0 default:
 *                     the device's), or force_tile_split 0 for results independent of the device
 *   "force_tail_exp":block pairs in spatial order: tile pairs whose boxes are >= r_t apart are
 *                     skipped with every ion's force kept within eps = 10^-k of the exact sum to
 *                     L/2 (g(r) = one pair's |F| at distance r, SpeedUp:224); k = 12 default, 0 =
 *                     exact (r_t = L/2); a no-op where the a-priori radius below is >= L/2 (every
 *                     BASELINE size but N ~ 1e6).  "force_skip_radius" reports r_t
 *   "force_tail_mode": how r_t is bounded.  1 (default, every world size) = measured and
 *                     enforced: r_t from a density model of the per-sub-tile sums (<= the a-priori
 *                     radius); every force call sums, per 16-ion sub-tile, n g(sub-box distance)
 *                     over the pairs it drops inside L/2 (all-reduced over the ranks), and every
 *                     tile with a sub-tile sum over eps gets its ions' forces recomputed exactly
 *                     (all pairs to L/2), so eps holds for any configuration; when that happened
 *                     the next host sync widens r_t (stderr says so).  "force_tail_bound" = the
 *                     largest sub-tile sum of the other tiles over the measured calls (NaN before
 *                     one; reset with new positions, N or these options — new positions of the same N
 *                     keep the widened r_t), "force_tail_raw_bound" the
 *                     largest of all, "force_tail_fixed_tiles" the tiles recomputed so far,
 *                     "force_tail_model_bound" the model's sum at r_t.  0 = a priori:
 *                     r_t the smallest radius with (N - 1) g(r_t) <= eps, "force_tail_bound" that
 *   "force_mid_exp":  block pairs in spatial order: 16-ion sub-tile groups >= r_mid apart take the
 *                     mid pair form (rsq + one Newton step, table 2^t with a degree-4 series; a
 *                     term within (r/lDeb + 3)(2.2e-14 + 2^-52) + 4e-15 relative), r_mid the
 *                     smallest radius with (N - 1) g(r) err(r) <= 10^-k; k = 13 default, 0 = off.
 *                     "force_mid_radius" / "force_mid_bound"
 *   "force_far_exp":  block pairs in spatial order: tile pairs >= r_far apart evaluate their pairs
 *                     within 3e-9 relative (rsq + one Newton step, degree-6 2^f), r_far the
 *                     smallest radius with (N - 1) g(r_far) 3e-9 <= 10^-k: every ion's force
 *                     within 10^-k more; k = 13 default, 0 = off.  "force_far_radius" /
 *                     "force_far_bound" report r_far and the bound
 *   "force_vfar_exp": the very-far form beyond r_vfar (raw v_rsq_f64, degree-5 2^f; its error
 *                     (r/lDeb + 3) 2^-23 + 1.1e-7 relative): (N - 1) g(r) err(r) <= 10^-k; k = 13
 *                     default, 0 = off.  "force_vfar_radius" / "force_vfar_bound"
 *   "force_ufar_exp": the ultra-far forms: beyond r_ufar the raw rsq and 2^t by v_exp_f32, and
 *                     beyond r_ufar32 (uniform-image tile pairs, only while the cutoff's own term
 *                     (N - 1) g(L/2 (1 - 2^-20)) stays inside the budget) the pair terms in f32;
 *                     each shell's bound <= 10^-k; k = 13 default, 0 = off.  "force_ufar_radius",
 *                     "force_ufar32_radius", "force_ufar_bound" (both shells)
 *   "force_form_mode": how the four tiers' radii are bounded (round 6).  1 (default, with
 *                     force_tail_mode 1, spatial order and the fast variant) = measured and
 *                     enforced: every force call's per-sub-tile sums also hold, for each sub-block
 *                     evaluated in an error-bounded form, n g(gap) err_form(gap); they are held to
 *                     "force_error_eps" (the tail's eps where r_t < L/2, + 10^-k per active tier) and
 *                     a tile over it is recomputed exactly, as for the tail; the radii come from a
 *                     density model of those sums (<= the a-priori radii) and widen with r_t when a
 *                     configuration exceeded it; the f32 form only for groups whose pairs are all
 *                     closer than L/2 (1 - 2^-20).  "force_tail_bound" is then the measured bound on
 *                     every ion's total deviation from the exact sum to L/2, the *_bound
 *                     constants the model's; "force_form_measured" 1 where mode 1 applies.  2 = as
 *                     1, and where the tail skips nothing (r_t = L/2) the active tiers share its
 *                     unused 10^-force_tail_exp equally (each tier's eps 10^-k + that share), so
 *                     every configuration's per-ion total is the one an active tail has.  0 = the
 *                     a-priori radii above
 *   "qt_enabled":     1 = qstep() runs in the substeps, 0 = skipped (t still advances): the
 *                     pumping programs' pump window (randomFrozenStartTag408Linear.cpp main)
 *   "qt_math":        0 = the reference's exact operations, 1 = FMA-contracted with a refined
 *                     rsq for 1/sqrt(1-dp), 2 = reassociated (default: fixed FMA chains per row
 *                     of M, folded constants; ~3x fewer instructions per substep).  1 and 2
 *                     differ from 0 by rounding only (1e-12 qstep gate); substep_kernel settings
 *                     are bit-identical to each other within one qt_math mode
 *   "qt_im01":        1 (default where the table allows) = the lane kernel's production launch
 *                     drops the real-part FMAs of the purely imaginary static coupling slots,
 *                     0 = the general instance (bit-identical up to the sign of zero)
 *   "potential_n3":   1 (default) = Epotential on the Newton-3 tiles / blocks (each distinct
 *                     pair once; world 1), 0 = the owner-computes potential rows (Epot within 1e-14 relative)
 *   "potential_plan": Newton-3 blocks (N > 65,536, world 1): 1 (default, round 6) = Epotential on the
 *                     force call's plan — its skip radius, sub-tile groups, error-bounded pair forms and
 *                     enforced tail; u(r) < lDeb g(r), so every U_i is within lDeb x the force call's
 *                     per-ion bound (~1e-12) of its sum to L/2; 0 = every pair to L/2 in the exact form
 *   "init_threads":   init() rejection sampling: 0 = auto, 1 = sequential, k = k host threads
 *                     (bit-identical positions, psi and drand48 state in every setting)
 *   "fused_step", "overlap": 1 = the one-launch MD step / the two-stream MD step (measured and
 *                     kept off by default; bit-identical to 0)
 *   "expt_force_sig": diagnostic only (force launches with arrival counts, no consumer) */
int         mdqt_set_option(mdqt_ctx* c, const char* name, int value);

/* ---- streams, timing, multi-GPU plumbing ---- */
int         mdqt_set_stream(mdqt_ctx* c, void* hip_stream);  /* NULL = the context's own stream */
void*       mdqt_get_stream(mdqt_ctx* c);
int         mdqt_synchronize(mdqt_ctx* c);
/* slab of rank r: ions [lo, hi) with slab capacity S = ceil(N / world) (pure function) */
int         mdqt_slab(int N, int world, int rank, int* lo, int* hi, int* S);
/* device address of the gathered position array [world][3][S] (doubles) and S */
int         mdqt_positions_device(mdqt_ctx* c, void** dptr, int* S);
int         mdqt_slab_bounds(const mdqt_ctx* c, int* lo, int* hi);
int         mdqt_set_counters(mdqt_ctx* c, int c0, unsigned counter, double Epot, double Epot0);
/* RCCL (one process per GPU).  Rank 0 makes the 128-byte unique id, the launcher
 * broadcasts it (torch.distributed), every rank calls mdqt_comm_init.  With a communicator,
 * mdqt_md_steps / mdqt_run all-gather the position slabs (in place, [world][3][S]) before
 * every force call, and epotential / observables / output / write_conditions become
 * collectives (sum all-reduces; rank 0 writes the files). */
int         mdqt_comm_unique_id(void* out, size_t len);
int         mdqt_comm_init(mdqt_ctx* c, const void* uid, size_t len);
/* ranks in this context's communicator: ncclCommCount of the RCCL communicator, the group size
 * of an in-process group, 1 without either (the bench checks it against --gpus) */
int         mdqt_comm_size(const mdqt_ctx* c, int* n);
/* in-process group of world_size contexts (tests on one GPU): the all-gather becomes device
 * copies; the caller steps the ranks in lockstep (all all-gathers, then all forces ...) */
int         mdqt_comm_init_local(mdqt_ctx* const* ctxs, int n);
int         mdqt_allgather_positions(mdqt_ctx* c);
int         mdqt_allreduce_sum(mdqt_ctx* c, double* host_buf, size_t n);
/* Per-rank partial sums for output() under sharding: out[0] = sum vx, [1..3] = sum of the
 * reference's EkinX/Y/Z terms about vxAvg, [4] = sum over owned i of the full-row pair
 * potential, Pvel partial [3][2001] before normalisation.  Used by the sharded driver. */
int         mdqt_partial_observables(mdqt_ctx* c, double vxAvg, double out5[5], double* Pvel_partial);
/* kernel timing: with period k > 0, every k-th force launch and every k-th fused-substep
 * launch is bracketed by HIP events on the context stream (k = 1: all; 0: off); totals()
 * syncs, returns the summed device time (ms) and bracketed-launch counts since the last
 * call, and resets. */
int         mdqt_enable_timing(mdqt_ctx* c, int period);
/* the same for one kind only: kinds bit 0 = force launches, bit 1 = fused-substep launches (an
 * event-timed launch costs its MD step a few us, so a timed region may sample only its dominant
 * kernel) */
int         mdqt_enable_timing_kinds(mdqt_ctx* c, int period, int kinds);
/* the same with the bracketed launches at index `offset` mod period (0 <= offset < period;
 * enable_timing_kinds takes period / 2) */
int         mdqt_enable_timing_at(mdqt_ctx* c, int period, int kinds, int offset);
/* the Newton-3 block kernel's evaluated lane-steps per block of this rank (every tile-pair class but the
 * skipped ones) for the current positions: out[0 .. *nblocks) for blocks Plo .. Phi - 1; at world 1
 * every block, so the work of any partition of the blocks over ranks follows (load balance) */
int         mdqt_force_block_work(mdqt_ctx* c, double* out, int n, int* nblocks);
/* the block kernel's lock-step J loop for the current positions (diagnostic): out[0] the estimated VALU
 * instructions of all its tile pairs (per-form counts), out[1] 8 x the sum over J steps of the busiest
 * wave's, out[2] the J steps with work; out[1] / out[0] = the max-over-mean excess the J-step barriers cost */
int         mdqt_force_jstep_balance(mdqt_ctx* c, double* out, int n);
/* force_form_mode 1's tier radius for given parameters, without a context (host arithmetic only, for
 * tests): level 1 far, 2 very far, 3 ultra far, 4 ultra far in f32, 5 mid; k the tier's exponent (eps =
 * 10^-k); hi the skip radius the density model integrates to (L/2 without a tail); scale the model's
 * scale (1 until a configuration exceeded its bound).  apriori 0: the model radius (the smallest r with
 * 1.25 scale rho int_r^hi 4 pi (x + delta)^2 g(x) err(x) dx <= eps, capped by the a-priori radius);
 * 1: force_form_mode 0's a-priori radius ((N - 1) g(r) err(r) <= eps, + the f32 tier's cutoff term);
 * 2: the a-priori radius without that term.  *radius = L/2 when the tier is off; *bound its bound. */
int         mdqt_tier_radius_model(int N, double L, double lDeb, int k, int level, double hi, double scale,
                                   int apriori, double* radius, double* bound);
int         mdqt_kernel_time_totals(mdqt_ctx* c, double* force_ms, int* nforce, double* substep_ms,
                                    int* nsub);
/* the same with the Newton-3 block kernel (k_pairs_n3b, N > 65,536) timed on its own inside every
 * timed force call (its dispatch timestamps: the plan, the slot reduction, the tail pass and the
 * collectives excluded): out[6] = force_ms, n_force, substep_ms, n_substep, block_ms, n_block */
int         mdqt_kernel_times(mdqt_ctx* c, double* out, int n);
/* with n >= 8, out[6..7] = the block kernel of the timed potential calls (Epotential on the Newton-3
 * blocks; timing kinds bit 2): ms, calls */
/* the force-call breakdown (timing kinds bit 3 with bit 0; block scheme, N > 65,536): since the last call,
 * the average ms per timed force call of out[0] the position all-gather just before it (0 at world 1),
 * [1] the spatial sort and boxes, [2] the plan, [3] the block kernel, [4] the slot reduction, [5] the tail
 * pass (all-reduce of the per-sub-tile sums, list, exact fix), [6] the reduce-scatter, [7] forces() from
 * start to end (= [1] + ... + [6]); out[8] = the timed calls.  Events between the stages on the context
 * stream; resets.  Replaces no reference function (measurement) */
int         mdqt_force_breakdown(mdqt_ctx* c, double* out, int n);

#ifdef __cplusplus
}
#endif
#endif /* MDQT_H */
