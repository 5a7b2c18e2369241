/*
 * ORACLE — TEST INFRASTRUCTURE ONLY.  Never linked into, loaded by, or called from the
 * product path (mdqtplasmasims_amd/).  Only tests/, __graft_entry__.smoke() and bench.py's
 * cpu_baseline leg may use it, and only as the checker / the timed CPU baseline.
 *
 * Plain-C restatement of the hot path of the reference program
 *   /root/reference/laserCoolingPlusExpansionMDQTSpeedUp.cpp   ("SpeedUp" below)
 * following its algorithm and its floating-point operation order line by line
 * (file:line citations next to every function in mdqt_oracle.c).
 *
 * Parity pinning:
 *   - drand48 stream: pinned bit-exactly against glibc's own srand48/drand48
 *     (tests/test_oracle_rng.py).
 *   - Yukawa force law, minimum image, cutoff, pair potential: pinned against the reference's
 *     own compiled code — MonteCarloFollowedByMDAndTempAnisotropy.cpp calculateAccelerations /
 *     calcUIJ (:387-448, :161-169), built unmodified by oracle/ref/Makefile into oracle/_ref/,
 *     and against the golden vectors it produced (tests/golden/).
 *   - Per-ion quantum-trajectory step (qstep, SpeedUp:438-717): PARITY UNPINNED against the
 *     reference — SpeedUp needs Armadillo 7.600.1, which is absent from this image, so the
 *     reference cannot be built here.  The restatement is cross-checked only against an
 *     independent literal dense transcription of the Armadillo algebra (tests/dense_qt.py)
 *     and analytic known-answer tests.
 */
#ifndef MDQT_ORACLE_H
#define MDQT_ORACLE_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* Reference user inputs (SpeedUp:56-85) plus the extensions the build needs. */
typedef struct orc_params {
    double Ge;            /* SpeedUp:60  kappa = sqrt(3*Ge)                         */
    double tmax;          /* SpeedUp:63  #define tmax 30                            */
    double density;       /* SpeedUp:65  units of 1e14 m^-3                          */
    double sig0;          /* SpeedUp:66                                              */
    double Te;            /* SpeedUp:67                                              */
    double fracOfSig;     /* SpeedUp:68                                              */
    double detuning;      /* SpeedUp:70                                              */
    double detuningDP;    /* SpeedUp:71                                              */
    double Om;            /* SpeedUp:72                                              */
    double OmDP;          /* SpeedUp:73                                              */
    int N0;               /* SpeedUp:69  #define N0 3500                            */
    int newRun;           /* SpeedUp:61                                              */
    int c0;               /* SpeedUp:62                                              */
    int sampleFreq;       /* SpeedUp:78                                              */
    int reNormalizewvFns; /* SpeedUp:74                                              */
    /* extensions */
    int qt_enabled;       /* 1 = MDQT (reference); 0 = MD-only: qstep body skipped, t advances */
    int rng_mode;         /* 0 = drand48 in reference order; 1 = Philox4x32-10 per (ion, qstep) */
    uint32_t seed;        /* value given to srand48 (reference: time(NULL)+job, SpeedUp:1219) */
    uint32_t job;         /* SpeedUp:1145 */
    int nthreads;         /* OpenMP threads for the race-free parallel loops (1 = serial) */
    int qt_model;         /* 0 = SpeedUp 12-level cooling; 1/2/3 = 408 linear / 408 quad / 422 linear
                           * optical pumping (randomFrozenStartTag*.cpp qstep; Philox only) */
    char saveDirectory[256]; /* SpeedUp:56 */
    double tpumpreal;     /* randomFrozenStartTag408Linear.cpp:58 (orc_run_pump) */
    double tstartV0;      /* randomFrozenStartTag408Linear.cpp:78 */
} orc_params;

typedef struct orc_sim orc_sim;

void   orc_default_params(orc_params* p);
orc_sim* orc_create(const orc_params* p);
void   orc_destroy(orc_sim* s);

/* derived constants (SpeedUp:79-85, :146-149, :295-297, :1181-1215) */
double orc_get_const(const orc_sim* s, const char* name);

/* SpeedUp:289-348 init(): drand48 rejection sampling of positions + random S superposition */
int    orc_init(orc_sim* s);

/* state access; R,V,F are [3][ld] row-major (the reference's R[3][N0+1000] layout);
 * psi is [N][12][2] interleaved (re,im) = cx_mat wvFns[] storage order. */
int    orc_get_N(const orc_sim* s);
void   orc_set_state(orc_sim* s, int N, const double* R, const double* V, size_t ld,
                     const double* psi, const double* tPart, double t);
void   orc_get_state(const orc_sim* s, double* R, double* V, double* F, size_t ld,
                     double* psi, double* tPart, double* t);
void   orc_set_forces(orc_sim* s, const double* F, size_t ld);
double orc_get_time(const orc_sim* s);
void   orc_set_time(orc_sim* s, double t);
void   orc_set_qt_constants(orc_sim* s, double dtQ, double gamToE, double pv2q, double r);
uint64_t orc_get_qstep_index(const orc_sim* s);
void   orc_set_qstep_index(orc_sim* s, uint64_t q);
void   orc_set_drand48_state(orc_sim* s, uint64_t x);
uint64_t orc_get_drand48_state(const orc_sim* s);
int    orc_get_counters(const orc_sim* s, int* c0, unsigned* counter, double* Epot, double* Epot0);

/* SpeedUp:192-236 forces() on the simulation state */
void   orc_forces(orc_sim* s);
/* Same force law on caller arrays (for cross-checks against the reference build):
 * F_i = sum_{j != i, ascending} f(i,j); R and F are [3][ld]. */
void   orc_forces_raw(int N, double L, double lDeb, const double* R, size_t ld, double* F, int nthreads);
/* owner-computes slab [lo,hi) of the same (for the sharding partition-invariance tests) */
void   orc_forces_rows(int N, int lo, int hi, double L, double lDeb, const double* R, size_t ld,
                       double* F, int nthreads);
/* rows idx[0..nidx) of the same pair terms, compensated (Neumaier) sum, F is [3][nidx] (sampled-ion
 * checks at large N) */
void   orc_forces_index(int N, double L, double lDeb, const double* R, size_t ld, const int* idx, int nidx,
                        double* F, int nthreads);
/* rows idx[0..nidx) of the pair potential (the terms of Epotential(), SpeedUp:256-266), compensated sum:
 * U[k] = sum over j != idx[k] inside L/2 of exp(-r/lDeb)/r */
void   orc_potentials_index(int N, double L, double lDeb, const double* R, size_t ld, const int* idx, int nidx,
                            double* U, int nthreads);
/* Philox ion key of local ion i = ids[i] (default i): a subset of a large system's ions run by the
 * oracle draws the same uniforms as the full system */
void   orc_set_ion_ids(orc_sim* s, const uint64_t* ids, int n);
/* SpeedUp:244-281 Epotential() (serial, reference order) */
double orc_epotential(orc_sim* s);
double orc_epotential_raw(int N, double L, double lDeb, const double* R, size_t ld);
/* SpeedUp:418-430 step(), SpeedUp:438-717 qstep() */
void   orc_step(orc_sim* s);
void   orc_qstep(orc_sim* s);
/* n x (step(); qstep()) with F frozen (the body of the time loop between forces() calls) */
void   orc_substeps(orc_sim* s, int n);
/* n x (forces(); ratio x (step(); qstep())) — MD steps as the time loop runs them */
void   orc_md_steps(orc_sim* s, int n);

/* SpeedUp:917-1032 observables of output(): returns EkinX,EkinY,EkinZ,Epot,Etot-Epot0,<vx>;
 * Pvel is [3][2001] (may be NULL), pops is [N][3] (S,P,D; may be NULL). */
void   orc_observables(orc_sim* s, double out7[7], double* Pvel, double* pops);

/* The full reference program flow (main, SpeedUp:1139-1383) writing the reference's
 * directory tree and files.  Returns 0 on success. */
int    orc_run(orc_sim* s);
int    orc_output(orc_sim* s);                 /* SpeedUp:917-1032 */
int    orc_write_conditions(orc_sim* s, int c0); /* SpeedUp:725-784 */
int    orc_read_conditions(orc_sim* s, int c0);  /* SpeedUp:785-916 */
int    orc_setup_directories(orc_sim* s);        /* SpeedUp:1145-1160 */
/* the optical-pumping programs' main() (randomFrozenStartTag408Linear.cpp:981-1076 and the 408Quad /
 * 422Linear copies; qt_model 1-3): leapfrog MD step every ratio quantum steps, qstep() only in
 * the pump window, measureSpinUps(), output() of the tagged ions, VAF, writeConditions() */
int    orc_run_pump(orc_sim* s);
/* its spin-up list (N ints) and count */
int    orc_get_spin_up_list(const orc_sim* s, int* tags);
const char* orc_save_directory(const orc_sim* s);

/* RNG primitives (exported for the known-answer tests) */
double orc_drand48_next(uint64_t* x);
uint64_t orc_srand48_state(uint32_t seed);
void   orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]);
double orc_philox_uniform(uint32_t seed, uint32_t job, uint64_t ion, uint64_t qstep, int draw);

/* single-ion qstep on explicit inputs (for the dense-transcription and KAT tests):
 * psi[24] in/out, *vx in/out (kick applied), *tPart in/out; u[5] are the uniforms u1..u5
 * the reference would draw (only u[0] used when no jump).  t is the global time used for the
 * expanding-frame detuning.  Returns 1 if a quantum jump occurred, 0 otherwise. */
/* spin-up tagging of the pumping models (measureSpinUps, randomFrozenStartTag408Linear.cpp:600,
 * randomFrozenStartTag422Linear.cpp:568): Philox draws 6 and 7 of (ion, current qstep index) */
int    orc_tag_spin_up(const orc_sim* s, int* tags);
int    orc_qstep_ion(const orc_sim* s, double t, double* psi, double* vx, double* tPart,
                     const double u[5], int* ndraws);

#ifdef __cplusplus
}
#endif
#endif
