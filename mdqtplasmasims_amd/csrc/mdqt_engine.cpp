// Host engine of the MI355X MDQT path: the C ABI of include/mdqt.h.
//
// Owns the device-resident state of one simulation (or one rank's slab of it), builds the
// reference's derived constants and QT operators, drives the gfx950 kernels of
// mdqt_kernels.hip on one HIP stream, and reproduces the reference program's control flow
// (main() time loop), initial conditions and text files.  Every function cites the lines of
// laserCoolingPlusExpansionMDQTSpeedUp.cpp ("SpeedUp") it stands in for.
#include <errno.h>
#include <math.h>
#include <stdarg.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include <string>
#include <algorithm>
#include <memory>
#include <thread>
#include <vector>

#include <rccl/rccl.h>

#include "../../include/mdqt.h"
#include "mdqt_internal.hpp"
#include "mdqt_writer.hpp"
#include "mdqt_init_sample.hpp"

using namespace mdqt;

namespace {

constexpr double TIMESTEP = 0.002;   // SpeedUp:80
constexpr int NINTERVALV = 13;       // numberOfIntervalV, SpeedUp:105

thread_local std::string g_err;

int fail(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return -1;
}

#define HIPCHK(expr)                                                                  \
    do {                                                                              \
        hipError_t e_ = (expr);                                                       \
        if (e_ != hipSuccess)                                                         \
            return fail("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__); \
    } while (0)

#define NCCLCHK(expr)                                                                   \
    do {                                                                                \
        ncclResult_t r_ = (expr);                                                       \
        if (r_ != ncclSuccess) return fail("%s failed: %s", #expr, ncclGetErrorString(r_)); \
    } while (0)

struct cx { double re, im; };
inline cx cx_make(double r, double i) { return {r, i}; }
inline cx cx_mul(cx a, cx b) { return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re}; }
inline cx cx_add(cx a, cx b) { return {a.re + b.re, a.im + b.im}; }
inline cx cx_sub(cx a, cx b) { return {a.re - b.re, a.im - b.im}; }
inline cx cx_conj(cx a) { return {a.re, -a.im}; }

// glibc drand48 (SpeedUp:303-333, srand48 :1219): mdqt_init_sample.hpp

}  // namespace

#ifndef MDQT_TAIL_MODE
#define MDQT_TAIL_MODE 1
#endif
#ifndef MDQT_FORM_MODE
#define MDQT_FORM_MODE 2
#endif
struct mdqt_ctx {
    mdqt_params p;
    // derived constants (SpeedUp:79-85, :146-149, :295-297)
    double gamToE, dtQ, pv2q, r, kRat, vKick, vKickDP, lDeb, L;
    int ratio;
    double gs[18];
    QTConst qc;
    double vel[NBINS];
    // sizes
    int N = 0, S = 0, lo = 0, hi = 0, nloc = 0;
    int capS = 0, capNseg = 0, nseg = 1, seglen = 1;
    // device
    int dev = 0;
    hipStream_t own = nullptr, stream = nullptr;
    double *dR = nullptr, *dV = nullptr, *dF = nullptr, *dFpart = nullptr, *dPsi = nullptr,
           *dTp = nullptr, *dScr = nullptr, *dKde = nullptr, *dUrow = nullptr;
    double* dUpart = nullptr;      // potential-row partials of its own (small systems, world 1)
    int n3_potential = 1;          // option "potential_n3": 1 = Newton-3 tiles where the forces use them
#ifndef MDQT_N3B_PAIRS_DEFAULT
#define MDQT_N3B_PAIRS_DEFAULT 1                  // A/B round 6 (r06e): N = 1M force call -4.3 %, C5 -2.3 %, C3 -2.3 %
#endif
    int n3b_pairs = MDQT_N3B_PAIRS_DEFAULT;   // option "force_n3b_pairs": the paired-wave block kernel (k_pairs_n3b_pw)
    int pot_plan = 1;              // option "potential_plan": 1 = Epotential on the blocks takes the force call's
                                   // plan (skips, sub-tile groups, error-bounded forms); 0 = every pair to L/2 exactly
    size_t capUpart = 0;
    double* dPack = nullptr;       // output()'s per-ion columns [4][S] (world 1)
    int kdeChunks = 0;
    LaneTab tab;                   // lane-per-state QT kernel tables (host copy)
    LaneTab* dTab = nullptr;       // device copy (uploaded once at create)
    FastTab ftab;                  // qt_math 2 row tables by state (host copy)
    FastTab ftabL;                 // the same by lane of the lane-per-state kernel (model 0: kStateOfLane0)
    FastTab* dFTab = nullptr;      // device copies [2]: by state, by lane
    int substep_mode = 0;          // 0 auto, 1 thread-per-ion, 2 lane-per-state
    int force_variant = 1;         // 0 exact reference operations, 1 fast reciprocal form
    int qt_math = 2;               // 0 exact reference operations, 1 FMA-contracted, 2 reassociated (option "qt_math")
    bool f_pending = false;        // dFpart holds unreduced force partials (pend_nseg > 1)
    int pend_nseg = 1;             // partial count of the pending forces (segments or slots)
    int scheme_opt = 0;            // force scheme: 0 auto, 1 rows (owner computes), 2 Newton-3 tiles, 3 Newton-3 blocks
    bool use_n3 = false;
    bool use_n3b = false;          // Newton-3 block pairs (k_pairs_n3b): large N, one GPU or sharded
    N3BArgs n3b;                   // its configuration (pointers and pair constants filled per call)
    double* dSlots = nullptr;      // its slots [nd + R][3][Npad]
    size_t capSlots = 0;
    double* dFr = nullptr;         // sharded n3b: this rank's dense partial forces [world][3][S]
    // spatial order of the n3b scheme (mdqt_sort.hip; option "force_sort", default on)
    int sort_mode = 1;             // 0 off, 1 sorted + tile-pair skipping, 2 sorted, nothing skipped (tests)
    int ax1_mode = 1;              // option "force_ax1": the one-axis per-pair image instance (1, auto) or not (0)
    // error-bounded force tail (option "force_tail_exp" k: eps = 10^-k, 0 = off): tile pairs whose
    // boxes are >= r_t apart are skipped, r_t the smallest radius with (N - 1) g(r_t) <= eps,
    // g(r) = (1/r + 1/lDeb) e^(-r/lDeb) / r the pair force magnitude (SpeedUp:224) — so no ion's
    // force changes by more than eps; a no-op where r_t >= L/2 (every BASELINE size but N ~ 1e6)
    int tail_exp = 12;
    // how r_t is bounded (option "force_tail_mode"): 0 a priori, (N - 1) g(r_t) <= eps; 1 (default,
    // every world size) measured and enforced: r_t from the density model's sum over tile pairs
    // (tail_radius_sum), every force call sums, per tile, n_J g(box distance) over its skipped tile
    // pairs on the device (k_pairs_n3b; all-reduced over the ranks), and every tile whose sum
    // exceeds eps gets the exact sum over those tile pairs added to its rows (k_tail_fix) — so every
    // ion meets eps whatever the configuration; the host widens r_t when that happened (tail_check)
    int tail_mode = MDQT_TAIL_MODE;
    double* dTail = nullptr;       // [4T]: the per-sub-tile sums of the current call
    unsigned long long* dTailSt = nullptr;   // [8]: k_tail_max's running maxima and counters
    int* dTailList = nullptr;      // [T]: this call's tiles over eps (this rank's)
    double tail_scale = 1.;        // r_t from 2 tail_scale B(r) <= eps: raised when a call exceeded eps
    unsigned long long tail_seen = 0;   // tiles over eps the host has reacted to
    int tail_warned = 0;                // stderr lines printed by tail_check
    bool tail_pending = false;     // in-process group: the sums wait for the group's (local_reduce)
    N3BArgs tail_args;             // ... with the call's arguments
    mutable double tail_key[5] = {0, 0, 0, 0, 0}, tail_val[2] = {0, 0};   // tail_radius_sum memo (N, L, lDeb, k, scale)
    // the far pair form (option "force_far_exp" k: eps = 10^-k, 0 = off): tile pairs whose boxes are
    // >= r_far apart evaluate their pairs within kFarRelErr (rsq1, degree-6 2^f), r_far the smallest
    // radius with (N - 1) g(r_far) kFarRelErr <= eps — so no ion's force moves by more than eps
    int far_exp = 13;
    // the mid pair form (round 4; option "force_mid_exp" k, 0 = off): sub-tile groups >= r_mid apart
    // take rsq1 and the table's 2^t with a degree-4 series, r_mid the smallest radius with (N - 1)
    // g(r_mid) ((r_mid/lDeb + 3)(kRsq1RelErr + 2^-52) + kTab4RelErr) <= 10^-k
    int mid_exp = 13;
    // the very-far pair form (option "force_vfar_exp" k, 0 = off): tile pairs >= r_vfar apart use
    // the raw rsq and a degree-5 2^f; r_vfar the smallest radius with
    // (N - 1) g(r) ((r/lDeb + 3) kRsqRawErr + kExp5RelErr) <= 10^-k
    int vfar_exp = 13;
    // the ultra-far pair form (option "force_ufar_exp" k, 0 = off): raw rsq and v_exp_f32, r_ufar the
    // smallest radius with (N - 1) g(r) ((r/lDeb) (kRsqRawErr + 2^-24) + 3 kRsqRawErr + kExp2fRelErr) <= 10^-k
    int ufar_exp = 13;
    // how the tiers' radii are bounded (option "force_form_mode", round 6): 0 a priori, (N - 1) g(r)
    // err(r) <= 10^-k per tier (far_radius_l); 1 (default, where the tail is measured: force_tail_mode 1,
    // spatial order, the fast variant) measured and enforced — every sub-block the plan evaluates in an
    // error-bounded form adds n_b g(gap) err_form(gap) to its sub-tiles' sums (k_n3b_plan), a tile whose
    // sum exceeds the call's eps (the tail's where r_t < L/2, + 10^-k per active tier: error_eps) is
    // recomputed exactly (k_tail_fix), and the radii come from the density model of those sums
    // (tier_radius) — so every ion meets that eps whatever the configuration; 2 as 1, and where the tail
    // is exact (r_t = L/2) the tiers share its unused 10^-tail_exp (tier_eps): the same total per ion
    int form_mode = MDQT_FORM_MODE;
    mutable double form_key[6][6] = {}, form_val[6][2] = {};   // tier_radius memo by level (N, L, lDeb, k, tail_exp, scale)
    uint32_t* dKeys = nullptr;     // [2][N] Hilbert keys, sorted keys
    int* dIon = nullptr;           // [2][N] identity, sorted index -> ion
    void* dSortTmp = nullptr;
    size_t sortTmpBytes = 0;
    double* dRs = nullptr;         // [3][Npad] positions in sorted order
    double* dBoxes = nullptr;      // [12][T] tile boxes, raw coordinate bounds
    double* dSubBoxes = nullptr;   // [6][4T] the 16-ion sub-tiles' boxes (the block kernel's sub-tile groups)
    uint2* dPlan = nullptr;        // [(Phi - Plo) nd][256] the block kernel's tile-pair words (k_n3b_plan)
    int tmask_mode = 1;            // option force_reduce_mask: k_n3b_reduce reads only the j-slots written
    int balance_opt = 1;           // option force_balance: sharded block ranges by census weight (1) or count (0)
    bool balanced = false;         // the block ranges of this N have been weighted (n3b_balance)
    double balance_ratio = NAN;    // max / mean of the ranks' evaluated lane-steps (the weighted ranges)
    double balance_ratio_eq = NAN; // the same for the equal-count ranges
    size_t capPlan = 0;
    int capSortN = 0;
    // overlapped MD step (option "overlap", OFF by default — measured slower): the
    // QT launch of step k runs on its own stream beside step k's force launch and waits on the
    // device for the force workgroups' arrivals (see md_steps_overlapped)
    int overlap_opt = 0;
    hipStream_t qs = nullptr;              // the QT stream
    hipEvent_t evQ = nullptr, evS = nullptr;
    unsigned long long* dArrive = nullptr; // [ntiles] finished tile pairs per tile, monotonic
    int arriveCap = 0;                     // tiles dArrive holds
    unsigned long long arriveEpoch = 0;    // each counter's value after the last launch (T per launch)
    // one MD step in one launch (option "fused_step", OFF by default — measured slower, DESIGN.md
    // §8): k_md_step, see md_step_fused
    int fused_opt = 0;
    int last_fused = 0;                    // the last MD step ran as one k_md_step launch
    int last_qt_kernel = 0;                // QT kernel instance of the last substep launch (QTKernel codes)
    int last_qt_nseg = 0;                  // force partials that launch summed in its prologue
    int* dSpinErr = nullptr;
    unsigned long long* force_arrive = nullptr;   // set around a force launch of an overlapped step
    hipStream_t sub_stream = nullptr;             // set around the QT launch of an overlapped step
    unsigned long long sub_target = 0;
    // the optical-pumping programs' main() (mdqt_run_pump)
    std::vector<int> spinUp;       // SpinUpList (randomFrozenStartTag408Linear.cpp:105)
    int nSpinUp = 0;
    int* dSpinUp = nullptr;        // device copy for the tagged distribution
    double* dTkde = nullptr;       // tagged KDE partials + result
    int pumpBin0 = -2000;          // velocity bins (j + pumpBin0) 0.0025: init() :306 / readConditions :723
    std::vector<double> vaHold;    // Vholder of Zfunc (:938-961)
    bool rs_pending = false;       // in-process group: F = sum of the ranks' dFr chunks, not formed yet
    const double** dPeerParts = nullptr;   // device array of the group's dFr pointers
    int nslots = 0, npairs = 0, capPairs = 0;
    int2* dPairs = nullptr;        // (I, J) tile pair of every wave of the Newton-3 kernel; after the
                                   // npairs entries, the split table (nsplit > 0: ensure_aux)
    int nsplit = 0;                // tile pairs the split table runs in parts (halves / quarters)
    int nsplit_wg = 0;             // workgroups of the split table
    int split_opt = 1;             // option force_tile_split: 0 off, 1 halves, 2 quarters (+ diagonal halves)
    int split_cus = 0;             // option force_split_cus: the CU count the split table is cut for (0: the device's)
    // rng_mode 0: the reference's drand48 stream, consumed in ion order on the device
    unsigned long long* dX48 = nullptr;   // [1] stream state + [48] jA + [48] jC
    int* dFlags = nullptr;         // [0] set by the substep kernels when a position leaves [-L/8, 9L/8]
    bool guard = false;            // host view: range-check every pair (see ForceArgs::guard)
    double* dU = nullptr;                 // [5][S] uniforms of the current substep
    ncclComm_t comm = nullptr;     // RCCL communicator over the world_size ranks (sharded runs)
    double* dComm = nullptr;       // device staging for small all-reduces
    std::vector<mdqt_ctx*> local;  // in-process group (tests on one GPU): all-gather by D2D copies
    size_t dCommCap = 0;
    // host-side state
    double t = 0.;
    uint64_t qidx = 0;
    int c0 = 0;
    unsigned counter = 0;
    double Epot = 0., Epot0 = 0.;
    uint64_t x48 = 0;
    std::vector<double> Vholder;   // [13][3][N] VZERO_* files (SpeedUp:752-763, :898-913)
    char saveDirectory[1024];
    std::unique_ptr<FileWriter> writer;   // background formatting/writing of the output files
    int init_threads = 0;          // init() sampling threads (option "init_threads"; 0 auto, 1 sequential)
    // timing
    // per-launch HIP events of the hot kernels (kind 0 = force, 1 = substeps), recorded on
    // the launch stream while timing is on; summed by mdqt_kernel_time_totals
    bool timing = false;
    unsigned tkinds = 3;                        // bit 0: force launches, bit 1: fused-substep launches
    unsigned tperiod = 1, tcount[2] = {0, 0};   // bracket launches k = toffset mod tperiod of each kind
    unsigned toffset = 0;                        // tperiod / 2 unless mdqt_enable_timing_at
                                                // (mid-period: not the first launch after a sync)
    std::vector<hipEvent_t> evpool[4];          // 2: the Newton-3 block kernel's own timestamps (a timed force call)
    int evused[4] = {0, 0, 0, 0};               // 3: the block kernel of the potential calls (Epotential on the blocks)
    // force-call breakdown (timing kind bit 3): per timed block-scheme force call the
    // events between its stages on the context stream — the preceding position all-gather (ag), then
    // m[0] start | sort + boxes | m[1] | plan | m[2] | block kernel | m[3] | slot reduction | m[4] |
    // tail pass (all-reduce, list, exact fix) | m[5] | reduce-scatter | m[6]
    struct BdCall { hipEvent_t ag0 = nullptr, ag1 = nullptr; hipEvent_t m[7] = {}; };
    std::vector<BdCall> bdcalls;
    std::vector<hipEvent_t> bdfree;
    hipEvent_t bd_ag[2] = {nullptr, nullptr};   // the all-gather just before the next timed force call
};

static int settle_forces(mdqt_ctx* s);
static int tail_check(mdqt_ctx* s);
static double u64_as_double(unsigned long long u) { double d; memcpy(&d, &u, sizeof d); return d; }

// force_tail_mode 1: forget what earlier calls measured (a new size or tail option).  keep_scale (new
// positions of the same system, e.g. a driver that uploads R every MD step): the statistics restart
// but the widened r_t stays — a clustered configuration does not rerun the exact pass, and warn, at
// every upload.  Callers settle pending forces first (they were measured with the old
// options: their enforcement must complete before the sums are cleared).
static int tail_reset(mdqt_ctx* s, bool keep_scale = false) {
    if (!keep_scale) s->tail_scale = 1.;
    s->tail_seen = 0;
    s->tail_pending = false;
    if (s->dTailSt) HIPCHK(hipMemsetAsync(s->dTailSt, 0, 16 * sizeof(unsigned long long), s->stream));
    return 0;
}

// The substep kernels raise dFlags[0] if a position leaves [-L/8, 9L/8] (an ion moving more than
// L/8 in half a substep: not a physical run).  Checked at every host synchronisation point;
// from then on every pair is range-checked, and the call reports the event as an error.
static int check_range_flag(mdqt_ctx* s) {
    if (s->dSpinErr) {                  // an overlapped QT launch gave up waiting for its forces
        int e = 0;
        if (hipMemcpyAsync(&e, s->dSpinErr, sizeof e, hipMemcpyDeviceToHost, s->stream) != hipSuccess ||
            hipStreamSynchronize(s->stream) != hipSuccess)
            return fail("reading the overlap flag failed");
        if (e) return fail("overlapped MD step: a QT launch timed out waiting for its force launch");
    }
    int f = 0;
    if (hipMemcpyAsync(&f, s->dFlags, sizeof f, hipMemcpyDeviceToHost, s->stream) != hipSuccess ||
        hipStreamSynchronize(s->stream) != hipSuccess)
        return fail("reading the position-range flag failed");
    if (f && !s->guard) {
        s->guard = true;
        return fail("positions left [-L/8, 9L/8] during the run (ion displacement > L/8 per half "
                    "substep); pair range checks are now on, but forces since the last sync used "
                    "the in-box minimum image");
    }
    return tail_check(s);
}

// ---------------------------------------------------------------------------------------------
// parameters and constants
// ---------------------------------------------------------------------------------------------

extern "C" void mdqt_default_params(mdqt_params* p) {
    memset(p, 0, sizeof(*p));
    p->Ge = 0.1; p->tmax = 30; p->density = 2; p->sig0 = 4.0; p->Te = 19.0; p->fracOfSig = 0;   // :60-68
    p->detuning = -1; p->detuningDP = 1; p->Om = 1; p->OmDP = 1;                               // :70-73
    p->N0 = 3500; p->newRun = 1; p->c0 = 0; p->sampleFreq = 40; p->reNormalizewvFns = 0;       // :61-78
    p->qt_enabled = 1; p->rng_mode = 1; p->seed = 12345; p->job = 1;
    p->device = -1; p->world_size = 1; p->rank = 0; p->force_segments = 0; p->qt_model = 0;
    strcpy(p->saveDirectory, "dataLaserCool/");                                              // :56
    p->tpumpreal = 0.0000002; p->tstartV0 = 15;           // randomFrozenStartTag408Linear.cpp:58, :78
}

// The optical-pumping programs' compile-time globals (randomFrozenStartTag408Linear.cpp:52-80,
// randomFrozenStartTag408Quad.cpp:55-81, randomFrozenStartTag422Linear.cpp:52-78): N0 3500,
// Ge 0.1, density 2, sampleFreq 40, tmax 25, tstartV0 15 in all three; per program the pump
// detuning, Rabi frequency, pump time and directory.
extern "C" void mdqt_default_params_pump(mdqt_params* p, int qt_model) {
    mdqt_default_params(p);
    p->qt_model = qt_model;
    p->tmax = 25; p->Ge = 0.1; p->density = 2; p->N0 = 3500; p->sampleFreq = 40; p->tstartV0 = 15;
    if (qt_model == 2) {
        p->detuning = 0; p->Om = 2; p->tpumpreal = 0.0000001; strcpy(p->saveDirectory, "data/");
    } else if (qt_model == 3) {
        p->detuning = -1; p->Om = 1.3; p->tpumpreal = 0.0000001; strcpy(p->saveDirectory, "data422/");
    } else {
        p->detuning = -2.5; p->Om = 0.7; p->tpumpreal = 0.0000002; strcpy(p->saveDirectory, "data408/");
    }
}

extern "C" const char* mdqt_last_error(void) { return g_err.c_str(); }

namespace mdqt {
int set_error(const char* fmt, ...) {
    char buf[1024];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(buf, sizeof buf, fmt, ap);
    va_end(ap);
    g_err = buf;
    return -1;
}
}  // namespace mdqt
extern "C" const char* mdqt_version(void) { return "mdqt-mi355x 0.1 (gfx950)"; }

extern "C" int mdqt_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

// FastTab of the optical-pumping models (qt_model 1..3).  Decay channels cs[j] = |a><b| with
// weights gs[j] (randomFrozenStartTag408Linear.cpp main :1000-1019; ...422Linear.cpp main):
// decayMatrix_bb = sum_j gs[j] over the channels leaving b, hamDecayTerm = -i/2 decayMatrix;
// H = detunings on the P levels (-det -/+ v_q, :439) + S-P couplings -Om/2 sqrt(gs[x]) |a><b|
// + h.c. (:438); M = I - i h H.  No optical kick, no time-dependent coupling.
static void build_pump_tables(const mdqt_params* p, QTConst& q, FastTab& f) {
    const double r = q.r, h = q.h;                             // decayRatio (408: 0.0617 :118; 422: 0.0754 :116)
    // channel j = |a_j><b_j|: 408 a = {0,0,0,1,1,1,6,6,6,6}, 422 a = {1,1,0,0,4,4}; only b enters D
    static const int B408[10] = {2, 3, 4, 3, 4, 5, 2, 3, 4, 5};
    const double G408[10] = {1, 2. / 3, 1. / 3, 1. / 3, 2. / 3, 1, r, r, r, r};
    static const int B422[6] = {2, 3, 3, 2, 2, 3};
    const double G422[6] = {2. / 3, 1. / 3, 2. / 3, 1. / 3, r, r};
    const int m = p->qt_model;
    const int nch = m == 3 ? 6 : 10;
    double D[NS] = {0.};
    for (int j = 0; j < nch; ++j) {
        const int b = m == 3 ? B422[j] : B408[j];
        D[b] += m == 3 ? G422[j] : G408[j];
    }
    // couplings (row, col, sqrt(gs) factor): |a><b| and its conjugate
    struct Cp { int a, b; double g; };
    Cp cp[4];
    int ncp = 0;
    if (m == 1) { cp[0] = {1, 3, G408[3]}; cp[1] = {1, 5, G408[5]}; cp[2] = {0, 2, G408[0]}; cp[3] = {0, 4, G408[2]}; ncp = 4; }
    if (m == 2) { cp[0] = {1, 5, G408[5]}; cp[1] = {0, 4, G408[2]}; ncp = 2; }
    if (m == 3) { cp[0] = {1, 2, G422[0]}; cp[1] = {0, 3, G422[2]}; ncp = 2; }
    memset(&f, 0, sizeof f);
    for (int k = 0; k < 16; ++k)
        for (int j = 0; j < 3; ++j) f.col[j][k] = k < NS ? kFastColM[m][k][j] : k;
    const int nst = kModelStates[m];
    const int nP = m == 3 ? 2 : 4;
    for (int k = 0; k < nst; ++k) {
        f.mre[k] = 1. + h * (-0.5 * D[k]);
        f.hdp[k] = h * D[k];
        double e1 = 0.;
        if (k >= 2 && k < 2 + nP) e1 = (k < 2 + nP / 2) ? -1. : 1.;   // right (-v) / left (+v) P levels
        const double e0 = (k >= 2 && k < 2 + nP) ? -p->detuning : 0.;
        f.mi0[k] = -(h * e0);
        f.mi1[k] = -(h * e1);
    }
    for (int c = 0; c < ncp; ++c) {
        const double v = (-p->Om / 2) * sqrt(cp[c].g);      // H_ab = H_ba = v; M = -i h v
        const int rc[2][2] = {{cp[c].a, cp[c].b}, {cp[c].b, cp[c].a}};
        for (const auto& e : rc)
            for (int j = 0; j < 3; ++j)
                if (kFastColM[m][e[0]][j] == e[1]) { f.cre[j][e[0]] = 0.; f.cim[j][e[0]] = -(h * v); }
    }
    f.cphi = 0.;
    q.kickS = q.kickD = 0.;
    q.vKick = q.vKickDP = 0.;
}

static void build_constants(mdqt_ctx* s) {
    const mdqt_params* p = &s->p;
    // SpeedUp :79-85, :146; the pumping programs' own constants: 408 nm
    // (randomFrozenStartTag408Linear.cpp:67-75, :118; 408Quad :69-77, :121: round, not ceil) and
    // 422 nm (randomFrozenStartTag422Linear.cpp:66-74, :116: gamma ratio .894, velocity .967, D/S 0.0754)
    const int m = p->qt_model;
    s->gamToE = m == 3 ? 174.07 * .894 / sqrt(p->density) : 174.07 / sqrt(p->density);
    s->ratio = m == 0   ? (int)ceil(34.81 / sqrt(p->density))
               : m == 3 ? (int)round(34.81 * .894 / sqrt(p->density))
                        : (int)round(34.81 / sqrt(p->density));
    s->dtQ = TIMESTEP / s->ratio;
    s->pv2q = m == 3 ? 1.1821 * pow(p->density, 1. / 6) * .967 : 1.1821 * pow(p->density, 1. / 6);
    s->r = m == 3 ? 0.0754 : 0.0617;
    s->kRat = 0.395;                                            // :147
    s->vKick = 0.001208 / s->pv2q;                              // :148
    s->vKickDP = s->vKick * s->kRat;                            // :149
    s->lDeb = 1. / sqrt(3. * p->Ge);                            // :295
    s->L = pow(p->N0 * 4. * M_PI / 3., 0.333333333);            // :297
    const double r = s->r;
    double* gs = s->gs;                                         // :1181-1198
    gs[0] = sqrt(1.); gs[1] = sqrt(2. / 3); gs[2] = sqrt(1. / 3); gs[3] = sqrt(2. / 3);
    gs[4] = sqrt(1. / 3); gs[5] = sqrt(1.);
    gs[6] = sqrt(r * 2. / 3); gs[7] = sqrt(r * 4. / 15); gs[8] = sqrt(r * 1. / 15);
    gs[9] = sqrt(r * 2. / 5); gs[10] = sqrt(r * 2. / 5); gs[11] = sqrt(r * 1. / 5);
    gs[12] = sqrt(r * 1. / 5); gs[13] = sqrt(r * 2. / 5); gs[14] = sqrt(r * 2. / 5);
    gs[15] = sqrt(r * 1. / 15); gs[16] = sqrt(r * 4. / 15); gs[17] = sqrt(r * 2. / 3);
    // cs[k] = |a><b| (0-based), :1163-1180
    static const int A[18] = {1, 1, 0, 0, 1, 0, 6, 7, 8, 7, 8, 9, 8, 9, 10, 9, 10, 11};
    static const int B[18] = {2, 3, 3, 4, 4, 5, 5, 5, 5, 4, 4, 4, 3, 3, 3, 2, 2, 2};
    cx decay[NS][NS], hamDecay[NS][NS], ham[NS][NS];
    memset(decay, 0, sizeof decay); memset(hamDecay, 0, sizeof hamDecay); memset(ham, 0, sizeof ham);
    for (int j = 0; j < 18; ++j) {                              // :1201-1204
        const int b = B[j];
        const double g2 = gs[j] * gs[j];
        hamDecay[b][b] = cx_sub(hamDecay[b][b], cx_make(0., 0.5 * g2));
        decay[b][b] = cx_add(decay[b][b], cx_make(g2, 0.));
    }
    for (int k = 0; k < 6; ++k)                                 // :1206-1210
        if (k != 1 && k != 3) {
            const double v = ((-1. * gs[k]) * p->Om) / 2;
            ham[B[k]][A[k]] = cx_add(ham[B[k]][A[k]], cx_make(v, 0.));
        }
    for (int k = 6; k < 18; ++k)                                // :1211-1215
        if (k != 8 && k != 11 && k != 7 && k != 10 && k != 13 && k != 16) {
            const double v = (((-1. * gs[k]) * p->OmDP) / 2) / sqrt(r);
            ham[B[k]][A[k]] = cx_add(ham[B[k]][A[k]], cx_make(v, 0.));
        }
    QTConst& q = s->qc;
    memset(&q, 0, sizeof q);
    q.dtQ = s->dtQ; q.gamToE = s->gamToE;
    q.h = s->dtQ * s->gamToE;                                   // :526, :530
    q.dtHalf = s->dtQ * s->gamToE / 2;                          // :525
    q.invh = 1. / (s->dtQ * s->gamToE);                         // :532
    q.pv2q = s->pv2q; q.kRat = s->kRat; q.r = r;
    q.det = p->detuning; q.detDP = p->detuningDP;
    q.kickS = 1 * s->vKick * p->Om;                             // :503
    q.kickD = s->vKickDP * (p->OmDP / r);
    q.vKick = s->vKick; q.vKickDP = s->vKickDP;
    q.pD = r / (r + 1);                                         // :589
    for (int k = 0; k < 4; ++k) {
        q.dP[k] = decay[2 + k][2 + k].re;
        q.hdP[k] = hamDecay[2 + k][2 + k].im;
    }
    q.a8 = ((p->OmDP / 2) * gs[8]) / sqrt(r);                   // :508
    q.a11 = ((p->OmDP / 2) * gs[11]) / sqrt(r);
    // static off-diagonal M = I - i h H entries, built exactly as the dense algebra does
    const cx sI = cx_make(0., s->dtQ * s->gamToE);
    for (int e = 0; e < NSTATIC; ++e) {
        const int a = kStaticRC[e][0], b = kStaticRC[e][1];
        cx h = cx_add(cx_add(cx_make(0., 0.), ham[a][b]), cx_conj(ham[b][a]));
        cx hamil = cx_add(h, hamDecay[a][b]);
        cx M = cx_sub(cx_make(0., 0.), cx_mul(sI, hamil));
        q.Mre[e] = M.re; q.Mim[e] = M.im;
    }
    q.thS3 = gs[2] * gs[2];                                     // :637-643
    q.thS4 = gs[4] * gs[4];                                     // :652-658
    q.thD[0][0] = gs[17] * gs[17] / r; q.thD[0][1] = gs[17] * gs[17] / r + gs[16] * gs[16] / r;   // :612-632
    q.thD[1][0] = gs[14] * gs[14] / r; q.thD[1][1] = gs[14] * gs[14] / r + gs[13] * gs[13] / r;   // :644-650
    q.thD[2][0] = gs[11] * gs[11] / r; q.thD[2][1] = gs[11] * gs[11] / r + gs[10] * gs[10] / r;   // :659-665
    q.thD[3][0] = gs[8] * gs[8] / r;   q.thD[3][1] = gs[8] * gs[8] / r + gs[7] * gs[7] / r;       // :675-697
    for (int k = 0; k < 18; ++k) q.gs[k] = gs[k];
    q.renorm = p->reNormalizewvFns;
    q.model = p->qt_model;
    q.seed = p->seed; q.job = p->job;
    for (int i = 0; i < NBINS; ++i) s->vel[i] = (double)i * 0.0025;   // :340-344
    // lane tables of the lane-per-state kernel: row k of M, slots A < B < C by column
    LaneTab& t = s->tab;
    memset(&t, 0, sizeof t);
    static const int cols[NS][3] = {{3, 5, -1}, {2, 4, -1}, {1, 9, 11}, {0, 8, 10}, {1, 7, 9}, {0, 6, 8},
                                    {5, -1, -1}, {4, -1, -1}, {3, 5, -1}, {2, 4, -1}, {3, -1, -1}, {2, -1, -1}};
    static const int order[NS] = {0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 2, 2};
    auto static_idx = [](int r, int c) {
        for (int e = 0; e < NSTATIC; ++e)
            if (kStaticRC[e][0] == r && kStaticRC[e][1] == c) return e;
        return -1;
    };
    for (int k = 0; k < 16; ++k) {
        t.colA[k] = t.colB[k] = t.colC[k] = 0;
        t.order[k] = 2;
    }
    for (int k = 0; k < NS; ++k) {
        t.order[k] = order[k];
        int* slot[3] = {&t.colA[k], &t.colB[k], &t.colC[k]};
        double* cre[3] = {&t.cAre[k], &t.cBre[k], &t.cCre[k]};
        double* cim[3] = {&t.cAim[k], &t.cBim[k], &t.cCim[k]};
        for (int j = 0; j < 3; ++j) {
            const int c = cols[k][j];
            if (c < 0) continue;
            *slot[j] = c;
            const int e = static_idx(k, c);
            if (e >= 0) { *cre[j] = q.Mre[e]; *cim[j] = q.Mim[e]; }
        }
        t.hasB[k] = cols[k][1] >= 0;
        t.hasC[k] = cols[k][2] >= 0;
        if (k >= 2 && k < 6) { t.dP[k] = q.dP[k - 2]; t.hd[k] = q.hdP[k - 2]; }
    }
    t.dynC[4] = 1; t.dynScale[4] = q.a11;      // M49
    t.dynC[5] = 1; t.dynScale[5] = q.a8;       // M58
    t.dynB[8] = 1; t.dynScale[8] = q.a8;       // M85
    t.dynB[9] = 1; t.dynScale[9] = q.a11;      // M94
    // kick weights: lane k multiplies rho_im(w_k, w_colA) by gA, rho_im(w_k, w_colB) by gB (:503)
    t.gA[1] = gs[0]; t.gA[0] = gs[2]; t.gB[1] = gs[4]; t.gB[0] = gs[5];
    t.gB[8] = gs[8]; t.gB[9] = gs[11]; t.gA[10] = gs[14]; t.gA[11] = gs[17];
    t.gA[6] = gs[6]; t.gA[7] = gs[9]; t.gA[8] = gs[12]; t.gA[9] = gs[15];
    // qt_math 2 tables (mdqt_qtfast.hip): slots of kFastCol, constants folded
    FastTab& f = s->ftab;
    memset(&f, 0, sizeof f);
    const double h = q.h;
    for (int k = 0; k < 16; ++k)
        for (int j = 0; j < 3; ++j) f.col[j][k] = k < NS ? kFastCol[k][j] : k;
    for (int k = 0; k < NS; ++k) {
        for (int j = 0; j < 3; ++j) {
            const int c = kFastCol[k][j];
            if (c == k || c >= NS) continue;       // unused slot
            const int e = static_idx(k, c);
            if (e >= 0) { f.cre[j][k] = q.Mre[e]; f.cim[j][k] = q.Mim[e]; }
        }
        const bool P = k >= 2 && k < 6;
        f.mre[k] = P ? 1. + h * q.hdP[k - 2] : 1.;
        f.hdp[k] = P ? h * q.dP[k - 2] : 0.;
        // E_k = e0 + e1 u (:506-510); Im M_kk = -h E_k
        double e0 = 0., e1 = 0.;
        if (k >= 2) e0 = (k < 6) ? -q.det : -q.det + q.detDP;
        if (k == 2 || k == 3) e1 = -1.;
        else if (k == 4 || k == 5) e1 = 1.;
        else if (k == 6 || k == 7) e1 = 1. - q.kRat;
        else if (k == 8 || k == 9) e1 = -(1. + q.kRat);
        else if (k >= 10) e1 = q.kRat - 1.;
        f.mi0[k] = -(h * e0);
        f.mi1[k] = -(h * e1);
    }
    // time-dependent slot 2: M85, M94 = h a {-sin, cos}; M58, M49 = h a {sin, cos} (:508)
    f.dms[8] = -(h * q.a8);  f.dmc[8] = h * q.a8;
    f.dms[9] = -(h * q.a11); f.dmc[9] = h * q.a11;
    f.dms[5] = h * q.a8;     f.dmc[5] = h * q.a8;
    f.dms[4] = h * q.a11;    f.dmc[4] = h * q.a11;
    // kick weights of Im(w_k conj(w_c)) (:503), scale kickS/kickD * dtQ * gamToE folded in
    const double kS = q.kickS * q.dtQ * q.gamToE, kD = q.kickD * q.dtQ * q.gamToE;
    struct KW { int row, col, g; double sgn, scale; };
    const KW kws[12] = {{1, 2, 0, 1., kS},  {0, 3, 2, 1., kS},  {1, 4, 4, -1., kS}, {0, 5, 5, -1., kS},
                        {8, 5, 8, 1., kD},  {9, 4, 11, 1., kD}, {10, 3, 14, 1., kD}, {11, 2, 17, 1., kD},
                        {6, 5, 6, -1., kD}, {7, 4, 9, -1., kD}, {8, 3, 12, -1., kD}, {9, 2, 15, -1., kD}};
    // Every coupling edge has exactly one P endpoint (S-P and P-D edges; each P level has three),
    // so each term sits on its P state's lane: Im(w_a conj(w_P)) = -Im(w_P conj(w_a)).  The kick
    // is then the sum over the four P lanes — the same broadcast pattern as dp, not a 16-lane tree.
    for (const KW& w : kws)
        for (int j = 0; j < 3; ++j)
            if (kFastCol[w.col][j] == w.row) f.kw[j][w.col] = -(w.sgn * (w.scale * gs[w.g]));
    f.cphi = 2. * (1. + q.kRat) * q.gamToE;
    if (p->qt_model != 0) build_pump_tables(p, q, f);
    f.dt2 = (0.5 * q.dtQ) * (0.5 * q.dtQ);
    for (int k = 0; k < 4; ++k) q.hdPh[k] = f.hdp[2 + k];
    // the lane-indexed copy: model 0 moves state kStateOfLane0[l] to lane l (its slots are DPP
    // moves, col unused: self); the pumping models keep lane = state
    FastTab& fl = s->ftabL;
    fl = f;
    // one substep's kick is the recoil (vKick or vKickDP) or the optical kick sum_j kw_j Im(w conj(w_j))
    // over the P lanes, |w| |w_j| <= 16 taken generously
    {
        double kw = 0.;
        for (int j = 0; j < 3; ++j)
            for (int k = 0; k < 16; ++k) kw += fabs(f.kw[j][k]);
        q.kickmax = fmax(fabs(q.vKick), fabs(q.vKickDP)) + 16. * kw;
    }
    q.im01 = 1;                                        // slots 0 and 1 purely imaginary (checked)
    for (int k = 0; k < 16; ++k)
        if (f.cre[0][k] != 0. || f.cre[1][k] != 0.) q.im01 = 0;
    if (p->qt_model == 0) {
        memset(&fl, 0, sizeof fl);
        fl.cphi = f.cphi; fl.dt2 = f.dt2;
        for (int l = 0; l < 16; ++l) {
            for (int j = 0; j < 3; ++j) fl.col[j][l] = l;
            const int k = state_of_lane0(l);
            if (k >= NS) continue;
            for (int j = 0; j < 3; ++j) {
                fl.cre[j][l] = f.cre[j][k]; fl.cim[j][l] = f.cim[j][k]; fl.kw[j][l] = f.kw[j][k];
            }
            fl.dms[l] = f.dms[k]; fl.dmc[l] = f.dmc[k]; fl.mre[l] = f.mre[k];
            fl.mi0[l] = f.mi0[k]; fl.mi1[l] = f.mi1[k]; fl.hdp[l] = f.hdp[k];
        }
    }
}

// QT constants and FastTab of a pumping model driven by another engine (the MC + MD tagging
// programs, include/mdmc.h): the model's couplings, decay and jump rule (build_pump_tables)
// with the caller's quantum time step, gamma and velocity conversion
namespace mdqt {
void build_pump_program(int model, double detuning, double Om, double dtQ, double gamToE, double pv2q,
                        double decayRatio, uint32_t seed, uint32_t job, QTConst& q, FastTab& f) {
    memset(&q, 0, sizeof q);
    q.dtQ = dtQ; q.gamToE = gamToE;
    q.h = dtQ * gamToE;
    q.dtHalf = dtQ * gamToE / 2;
    q.invh = 1. / (dtQ * gamToE);
    q.pv2q = pv2q; q.r = decayRatio;
    q.pD = decayRatio / (decayRatio + 1);
    q.det = detuning;
    q.model = model; q.seed = seed; q.job = job; q.renorm = 0;
    mdqt_params p;
    memset(&p, 0, sizeof p);
    p.qt_model = model; p.detuning = detuning; p.Om = Om;
    build_pump_tables(&p, q, f);
    f.dt2 = (0.5 * dtQ) * (0.5 * dtQ);
    for (int k = 0; k < 4; ++k) q.hdPh[k] = f.hdp[2 + k];
}
}  // namespace mdqt

static double expDetuning_of(const mdqt_params* p, double t) {   // :447
    return 0.0126 * p->fracOfSig * p->Te * t /
           (sqrt(p->density) * p->sig0 * sqrt(1 + 0.00014314 * t * t * p->Te / (p->density * p->sig0 * p->sig0)));
}

// ---------------------------------------------------------------------------------------------
// sizing and allocation
// ---------------------------------------------------------------------------------------------

extern "C" int mdqt_slab(int N, int world, int rank, int* lo, int* hi, int* S) {
    if (N < 0 || world < 1 || rank < 0 || rank >= world) return fail("mdqt_slab: bad arguments");
    int s = (N + world - 1) / world;
    s = ((s + 63) / 64) * 64;
    if (s == 0) s = 64;
    int l = rank * s; if (l > N) l = N;
    int h = (rank + 1) * s; if (h > N) h = N;
    if (lo) *lo = l;
    if (hi) *hi = h;
    if (S) *S = s;
    return 0;
}

// this rank's blocks [lo, hi) of the Newton-3 block kernel and its runs: up to 65,536 workgroups per rank
// (runs of one or a few block distances, dispatched run-major: a short last round; A/B with 8-tile
// blocks: N = 1M -1.2 % vs 16,384, C3 and C5 flat)
static void n3b_set_range(N3BArgs& b, int lo, int hi) {
    b.Plo = lo;
    b.Phi = hi;
    const int nblk = std::max(b.Phi - b.Plo, 1);
    static const int wg_target = [] {               // (A/B experiments: MDQT_N3B_WG workgroups per rank)
        const char* e = getenv("MDQT_N3B_WG");
        return e && atoi(e) > 0 ? atoi(e) : 65536;
    }();
    int R = std::min(b.nd, (wg_target + nblk - 1) / nblk);
    b.runlen = (b.nd + R - 1) / R;
    b.R = (b.nd + b.runlen - 1) / b.runlen;
}

// j segmentation of the force sum: a function of N only (partition invariance across world
// sizes); enough (row x segment) threads to fill 256 CUs at small N, segments >= 64 ions.
static void choose_segments(mdqt_ctx* s) {
    const int N = s->N;
    int nseg = s->p.force_segments;
    if (nseg <= 0) {
        const long target = 1L << 20;
        long a = (target + N - 1) / (N > 0 ? N : 1);
        long b = N / 64;
        nseg = (int)(a < b ? a : b);
        if (nseg < 1) nseg = 1;
    }
    if (nseg > N && N > 0) nseg = N;
    if (nseg < 1) nseg = 1;
    s->seglen = N > 0 ? (N + nseg - 1) / nseg : 1;
    s->nseg = N > 0 ? (N + s->seglen - 1) / s->seglen : 1;
    // Newton-3 tile pairs (one GPU, ntiles slots of 3 x S) up to 64k ions; above that Newton-3
    // block pairs (O(N^2/1024) slots, one GPU or sharded with a reduce-scatter); owner-computes
    // rows for small sharded systems (bit-identical across world sizes)
    const int W = s->p.world_size;
    int sch = s->scheme_opt;
    if (sch == 0) {
        if (W == 1) sch = N > 65536 ? 3 : (N >= 128 ? 2 : 1);
        else sch = N > 65536 ? 3 : 1;
    }
    s->use_n3 = sch == 2 && W == 1 && N >= 1;
    s->use_n3b = sch == 3 && N >= 1;
    const int nt = (N + 63) / 64;
    s->nslots = s->use_n3 ? nt : 0;
    s->npairs = s->use_n3 ? nt * (nt + 1) / 2 : 0;
    N3BArgs& b = s->n3b;
    memset(&b, 0, sizeof b);
    if (s->use_n3b) {
        b.N = N; b.T = nt; b.Npad = nt * 64;
        b.NB = (nt + kN3BBlock - 1) / kN3BBlock;
        b.nd = b.NB / 2 + 1;
        n3b_set_range(b, (int)((long)s->p.rank * b.NB / W), (int)((long)(s->p.rank + 1) * b.NB / W));
        s->balanced = false;
    }
}

// partial-sum buffer (row segments or Newton-3 slots) and the tile-pair table
// The tile kernel's last round of workgroups (C2: 1,596 on 256 CUs, 6 per CU and 60 more) decides
// its end: the 56 diagonal tile pairs (half the steps) go last already (the table below), and the
// split table also runs the 4 full tile pairs that remain in that round as two half workgroups each
// (the first / second 8 of every wave's 16 rotation steps) — 64 half-work workgroups in the last
// round instead of 56 + 4 whole ones, so no CU runs 7 whole tile pairs.  The second halves write
// their rows into one extra slot (ntiles; the split pairs have disjoint tiles, (0, 1), (2, 3), ...,
// and every other row of that slot stays 0), so F = the sum of ntiles + 1 slots.  The overlapped and
// fused MD steps (tile arrival counts) keep the plain table.
// Option 2 (quarters) runs those tile pairs in four parts and every diagonal tile in two: the last
// round is then 4 k + 2 nt quarter-size workgroups (C2: 128), so its CUs carry 6.25 tile pairs of work
// instead of 6.5 (measured: the same launch time as halves, profiles/r05n_tile_split_quarters_ab.txt).
// Extra slots: halves ntiles; quarters ntiles + 0 .. 2 (parts 1-3) and ntiles + 3 (diagonal halves).
static int split_slots(const mdqt_ctx* s) { return s->nsplit > 0 ? (s->split_opt == 2 ? 4 : 1) : 0; }
static int tile_split_count(const mdqt_ctx* s, int nt) {
    if (!s->split_opt || nt < 2) return 0;
    // the table (hence the summation order of the split tiles' forces, F's last bits) follows the CU count:
    // force_split_cus fixes it, so that devices with different counts give the same bits
    int ncu = s->split_cus;
    if (ncu <= 0 && (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, s->dev) != hipSuccess || ncu <= 0))
        return 0;
    const long w0 = (long)nt * (nt + 1) / 2;
    if (w0 <= ncu || w0 > 8L * ncu) return 0;    // one round (nothing to balance) / many (dispatched as CUs free up)
    const int k = (int)(w0 % ncu) - nt;          // whole tile pairs in the last round
    const int last = s->split_opt == 2 ? 4 * k + 2 * nt : 2 * k + nt;   // workgroups of the last round
    return (k > 0 && last <= ncu && 2 * k <= nt) ? k : 0;
}

static int ensure_aux(mdqt_ctx* s) {
    const int nt_split = (s->N + 63) / 64;
    s->nsplit = s->use_n3 && s->npairs > 0 ? tile_split_count(s, nt_split) : 0;
    const int need = std::max(std::max(s->nseg, s->nslots + split_slots(s)), 2);
    if (need > s->capNseg) {
        if (s->dFpart) HIPCHK(hipFree(s->dFpart));
        s->dFpart = nullptr;
        HIPCHK(hipMalloc(&s->dFpart, (size_t)s->capS * 3 * need * sizeof(double)));
        s->capNseg = need;
    }
    if (s->use_n3b) {
        const size_t need_s = (size_t)(s->n3b.nd + s->n3b.R) * 3 * s->n3b.Npad;
        if (need_s > s->capSlots) {
            if (s->dSlots) HIPCHK(hipFree(s->dSlots));
            s->dSlots = nullptr;
            HIPCHK(hipMalloc(&s->dSlots, need_s * sizeof(double)));
            s->capSlots = need_s;
        }
        if (s->p.world_size > 1 && !s->dFr)
            HIPCHK(hipMalloc(&s->dFr, (size_t)s->capS * 3 * s->p.world_size * sizeof(double)));
        if (s->sort_mode && s->N > s->capSortN) {
            for (void* q : {(void*)s->dKeys, (void*)s->dIon, s->dSortTmp, (void*)s->dRs, (void*)s->dBoxes,
                            (void*)s->dSubBoxes})
                if (q) HIPCHK(hipFree(q));
            s->dKeys = nullptr; s->dIon = nullptr; s->dSortTmp = nullptr; s->dRs = nullptr; s->dBoxes = nullptr;
            s->dSubBoxes = nullptr;
            const int Nc = s->N;
            const int Tc = (Nc + 63) / 64;
            HIPCHK(hipMalloc(&s->dKeys, (size_t)2 * Nc * sizeof(uint32_t)));
            HIPCHK(hipMalloc(&s->dIon, (size_t)2 * Nc * sizeof(int)));
            s->sortTmpBytes = spatial_order_tmp_bytes(Nc);
            if (!s->sortTmpBytes) return fail("radix sort scratch size query failed");
            HIPCHK(hipMalloc(&s->dSortTmp, s->sortTmpBytes));
            HIPCHK(hipMalloc(&s->dRs, (size_t)3 * Tc * 64 * sizeof(double)));
            HIPCHK(hipMalloc(&s->dBoxes, (size_t)12 * Tc * sizeof(double)));
            HIPCHK(hipMalloc(&s->dSubBoxes, (size_t)6 * 4 * Tc * sizeof(double)));
            if (s->dTail) HIPCHK(hipFree(s->dTail));
            if (s->dTailList) HIPCHK(hipFree(s->dTailList));
            s->dTail = nullptr; s->dTailList = nullptr;
            HIPCHK(hipMalloc(&s->dTail, (size_t)4 * Tc * sizeof(double)));
            HIPCHK(hipMemset(s->dTail, 0, (size_t)4 * Tc * sizeof(double)));
            HIPCHK(hipMalloc(&s->dTailList, (size_t)Tc * sizeof(int)));
            if (!s->dTailSt) {                       // [0, 8) the force calls', [8, 16) the potential calls'
                HIPCHK(hipMalloc(&s->dTailSt, 16 * sizeof(unsigned long long)));
                HIPCHK(hipMemset(s->dTailSt, 0, 16 * sizeof(unsigned long long)));
            }
            s->capSortN = Nc;
            if (tail_reset(s)) return -1;                // a new size: nothing measured yet
        }
    }
    if (s->use_n3 && s->npairs > 0) {
        const int tot = s->npairs + (s->nsplit > 0 ? s->npairs + 3 * s->nsplit + s->npairs : 0);   // (bound)
        if (tot > s->capPairs) {
            if (s->dPairs) HIPCHK(hipFree(s->dPairs));
            s->dPairs = nullptr;
            HIPCHK(hipMalloc(&s->dPairs, (size_t)tot * sizeof(int2)));
            s->capPairs = tot;
        }
        const int nt = (s->N + 63) / 64;
        std::vector<int2> h;
        h.reserve(s->npairs);
        // the diagonal tile pairs (half the rotation steps) last: they land in the dispatcher's
        // last round of workgroups, where the 7th workgroup of a CU goes (C2: 1,596 workgroups on
        // 256 CUs), so those CUs finish sooner (force launch 17.8 -> 17.3 us).  The slots a tile
        // pair writes do not depend on its position in the list: the same results.
        for (int I = 0; I < nt; ++I)
            for (int J = I + 1; J < nt; ++J) h.push_back(make_int2(I, J));
        for (int I = 0; I < nt; ++I) h.push_back(make_int2(I, I));
        if ((int)h.size() != s->npairs) return fail("tile-pair table size mismatch");
        if (s->nsplit > 0) {                         // the split table (tile_split_count)
            const int k = s->nsplit;
            auto split = [&](int I, int J) { return J == I + 1 && (I & 1) == 0 && I < 2 * k; };
            auto part = [](int I, int pl, int p) { return (int)(((unsigned)pl << 30) | ((unsigned)p << 28) | (unsigned)I); };
            for (int I = 0; I < nt; ++I)
                for (int J = I + 1; J < nt; ++J)
                    if (!split(I, J)) h.push_back(make_int2(I, J));
            if (s->split_opt == 2) {                 // quarters of the split pairs, halves of the diagonal tiles
                for (int p = 0; p < 4; ++p)
                    for (int m = 0; m < k; ++m) h.push_back(make_int2(part(2 * m, 2, p), 2 * m + 1));
                for (int p = 0; p < 2; ++p)
                    for (int I = 0; I < nt; ++I) h.push_back(make_int2(part(I, 1, p), I));
            } else {                                 // halves of the split pairs around the diagonal tiles
                for (int m = 0; m < k; ++m) h.push_back(make_int2(part(2 * m, 1, 0), 2 * m + 1));
                for (int I = 0; I < nt; ++I) h.push_back(make_int2(I, I));
                for (int m = 0; m < k; ++m) h.push_back(make_int2(part(2 * m, 1, 1), 2 * m + 1));
            }
            s->nsplit_wg = (int)h.size() - s->npairs;
            if (s->nsplit_wg != s->npairs + (s->split_opt == 2 ? 3 * k + nt : k)) return fail("split tile-pair table size mismatch");
            // the extra slots: only later parts of split tile pairs write them (their rows), every other row 0
            HIPCHK(hipMemsetAsync(s->dFpart + (size_t)nt * 3 * s->S, 0, (size_t)split_slots(s) * 3 * s->S * sizeof(double),
                                  s->stream));
        }
        HIPCHK(hipMemcpyAsync(s->dPairs, h.data(), h.size() * sizeof(int2), hipMemcpyHostToDevice, s->stream));
        HIPCHK(hipStreamSynchronize(s->stream));
    }
    return 0;
}

static void free_device(mdqt_ctx* s) {
    double** ps[] = {&s->dR, &s->dV, &s->dF, &s->dFpart, &s->dPsi, &s->dTp, &s->dScr, &s->dKde, &s->dUrow, &s->dU,
                     &s->dUpart, &s->dPack};
    for (double** q : ps) { if (*q) (void)hipFree(*q); *q = nullptr; }
    s->capUpart = 0;
    if (s->dPairs) (void)hipFree(s->dPairs);
    s->dPairs = nullptr;
    s->capPairs = 0;
    if (s->dSlots) (void)hipFree(s->dSlots);
    if (s->dFr) (void)hipFree(s->dFr);
    for (void* q : {(void*)s->dKeys, (void*)s->dIon, s->dSortTmp, (void*)s->dRs, (void*)s->dBoxes, (void*)s->dSubBoxes})
        if (q) (void)hipFree(q);
    s->dKeys = nullptr; s->dIon = nullptr; s->dSortTmp = nullptr; s->dRs = nullptr; s->dBoxes = nullptr;
    s->dSubBoxes = nullptr;
    if (s->dTail) (void)hipFree(s->dTail);
    if (s->dTailList) (void)hipFree(s->dTailList);
    if (s->dTailSt) (void)hipFree(s->dTailSt);
    s->dTail = nullptr; s->dTailList = nullptr; s->dTailSt = nullptr;
    s->capSortN = 0;
    if (s->dPlan) (void)hipFree(s->dPlan);
    s->dPlan = nullptr; s->capPlan = 0;
    if (s->dPeerParts) (void)hipFree((void*)s->dPeerParts);
    s->dSlots = nullptr; s->dFr = nullptr; s->dPeerParts = nullptr;
    s->capSlots = 0;
    s->capS = 0; s->capNseg = 0; s->kdeChunks = 0;
}

// (re)size everything for N ions; device contents are NOT preserved (callers upload after)
static int resize(mdqt_ctx* s, int N) {
    if (N < 0) return fail("negative N");
    int lo, hi, S;
    if (mdqt_slab(N, s->p.world_size, s->p.rank, &lo, &hi, &S)) return -1;
    s->N = N; s->lo = lo; s->hi = hi; s->nloc = hi - lo;
    choose_segments(s);
    const int W = s->p.world_size;
    if (S != s->capS) {
        free_device(s);
        HIPCHK(hipSetDevice(s->dev));
        const size_t sz = (size_t)S * sizeof(double);
        HIPCHK(hipMalloc(&s->dR, sz * 3 * W));
        HIPCHK(hipMalloc(&s->dV, sz * 3));
        HIPCHK(hipMalloc(&s->dF, sz * 3));
        HIPCHK(hipMalloc(&s->dPsi, sz * 24));
        HIPCHK(hipMalloc(&s->dTp, sz));
        HIPCHK(hipMalloc(&s->dUrow, sz));
        if (s->p.rng_mode == 0) HIPCHK(hipMalloc(&s->dU, sz * 5));
        HIPCHK(hipMalloc(&s->dScr, (64 + 3 * NBINS) * sizeof(double)));
        s->kdeChunks = 512;                            // chunks of >= 32 ions (the bins near v = 0 hold
        HIPCHK(hipMalloc(&s->dKde, (size_t)s->kdeChunks * 3 * NBINS * sizeof(double)));   // the work)
        HIPCHK(hipMalloc(&s->dPack, sz * 4));
        s->capS = S;
        HIPCHK(hipMemsetAsync(s->dR, 0, sz * 3 * W, s->stream));
        HIPCHK(hipMemsetAsync(s->dV, 0, sz * 3, s->stream));
        HIPCHK(hipMemsetAsync(s->dF, 0, sz * 3, s->stream));
        HIPCHK(hipMemsetAsync(s->dPsi, 0, sz * 24, s->stream));
        HIPCHK(hipMemsetAsync(s->dTp, 0, sz, s->stream));
    }
    s->S = S;
    if (ensure_aux(s)) return -1;
    s->Vholder.assign((size_t)NINTERVALV * 3 * (N > 0 ? N : 1), 0.);
    return 0;
}

extern "C" int mdqt_create(const mdqt_params* p, mdqt_ctx** out) {
    if (!p || !out) return fail("mdqt_create: NULL argument");
    *out = nullptr;
    if (p->rng_mode != 0 && p->rng_mode != 1)
        return fail("rng_mode must be 0 (drand48, reference order) or 1 (Philox)");
    if (p->rng_mode == 0 && p->world_size != 1)
        return fail("rng_mode 0 (one sequential drand48 stream) needs world_size 1");
    if (p->world_size < 1 || p->rank < 0 || p->rank >= p->world_size) return fail("bad world_size/rank");
    if (p->N0 < 1) return fail("N0 must be >= 1");
    if (p->sampleFreq < 1) return fail("sampleFreq must be >= 1");
    if (p->qt_model < 0 || p->qt_model >= NMODELS) return fail("qt_model must be 0..%d", NMODELS - 1);
    if (p->qt_model != 0 && p->rng_mode != 1)
        return fail("the optical-pumping qt_models run on the Philox stream (rng_mode 1)");
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev < 1) return fail("no HIP device available (%s)", hipGetErrorString(e));
    mdqt_ctx* s = new mdqt_ctx();
    s->p = *p;
    s->p.saveDirectory[sizeof(s->p.saveDirectory) - 1] = 0;
    if (p->device >= 0) {
        if (p->device >= ndev) { delete s; return fail("device %d >= device count %d", p->device, ndev); }
        s->dev = p->device;
    } else {
        (void)hipGetDevice(&s->dev);
    }
    if (hipSetDevice(s->dev) != hipSuccess || hipStreamCreateWithFlags(&s->own, hipStreamNonBlocking) != hipSuccess) {
        delete s;
        return fail("cannot create HIP stream on device %d", p->device);
    }
    s->stream = s->own;
    if (hipMalloc(&s->dTab, sizeof(LaneTab)) != hipSuccess || hipMalloc(&s->dFTab, 2 * sizeof(FastTab)) != hipSuccess) {
        mdqt_destroy(s);
        return fail("hipMalloc lane tables");
    }
    {
        const int f[2] = {0, 1};
        if (hipMalloc(&s->dFlags, sizeof f) != hipSuccess ||
            hipMemcpy(s->dFlags, f, sizeof f, hipMemcpyHostToDevice) != hipSuccess) {
            mdqt_destroy(s);
            return fail("hipMalloc flags");
        }
    }
    build_constants(s);
    if (s->p.rng_mode == 0) {
        unsigned long long h[97];
        h[0] = srand48_state(s->p.seed);
        unsigned long long A = 0x5DEECE66Dull, Cc = 0xBull;
        for (int b = 0; b < 48; ++b) {            // 2^b steps of X' = A X + C (mod 2^48)
            h[1 + b] = A; h[49 + b] = Cc;
            Cc = (A * Cc + Cc) & 0xFFFFFFFFFFFFull;
            A = (A * A) & 0xFFFFFFFFFFFFull;
        }
        if (hipMalloc(&s->dX48, sizeof h) != hipSuccess ||
            hipMemcpy(s->dX48, h, sizeof h, hipMemcpyHostToDevice) != hipSuccess) {
            mdqt_destroy(s);
            return fail("drand48 state upload failed");
        }
    }
    if (hipMemcpy(s->dTab, &s->tab, sizeof(LaneTab), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(s->dFTab, &s->ftab, sizeof(FastTab), hipMemcpyHostToDevice) != hipSuccess ||
        hipMemcpy(s->dFTab + 1, &s->ftabL, sizeof(FastTab), hipMemcpyHostToDevice) != hipSuccess) {
        mdqt_destroy(s);
        return fail("upload of the lane table failed");
    }
    s->t = 0.; s->qidx = 0; s->c0 = p->c0; s->counter = 0;
    s->x48 = srand48_state(p->seed);
    strncpy(s->saveDirectory, s->p.saveDirectory, sizeof(s->saveDirectory) - 1);
    s->saveDirectory[sizeof(s->saveDirectory) - 1] = 0;
    if (resize(s, 0)) { mdqt_destroy(s); return -1; }
    *out = s;
    return 0;
}

extern "C" void mdqt_destroy(mdqt_ctx* s) {
    if (!s) return;
    s->writer.reset();                                   // joins the file writers
    (void)hipSetDevice(s->dev);
    if (s->stream) (void)hipStreamSynchronize(s->stream);
    free_device(s);
    if (s->dTab) (void)hipFree(s->dTab);
    if (s->dFTab) (void)hipFree(s->dFTab);
    if (s->dComm) (void)hipFree(s->dComm);
    if (s->dSpinUp) (void)hipFree(s->dSpinUp);
    if (s->dArrive) (void)hipFree(s->dArrive);
    if (s->dSpinErr) (void)hipFree(s->dSpinErr);
    if (s->evQ) (void)hipEventDestroy(s->evQ);
    if (s->evS) (void)hipEventDestroy(s->evS);
    if (s->qs) (void)hipStreamDestroy(s->qs);
    if (s->dTkde) (void)hipFree(s->dTkde);
    if (s->dX48) (void)hipFree(s->dX48);
    if (s->dFlags) (void)hipFree(s->dFlags);
    if (s->comm) (void)ncclCommDestroy(s->comm);
    for (auto& pool : s->evpool)
        for (hipEvent_t ev : pool) (void)hipEventDestroy(ev);
    for (auto& c : s->bdcalls) {
        for (hipEvent_t ev : c.m) if (ev) (void)hipEventDestroy(ev);
        if (c.ag0) (void)hipEventDestroy(c.ag0);
        if (c.ag1) (void)hipEventDestroy(c.ag1);
    }
    for (hipEvent_t ev : s->bdfree) (void)hipEventDestroy(ev);
    for (hipEvent_t ev : s->bd_ag) if (ev) (void)hipEventDestroy(ev);
    if (s->own) (void)hipStreamDestroy(s->own);
    delete s;
}

static double tail_radius(int N, double L, double lDeb, int k, double* bound);
static double tail_radius_sum(const mdqt_ctx* s, double* bound);
static bool tail_measured(const mdqt_ctx* s);
static double skip_radius(const mdqt_ctx* s, double* bound);
static double far_radius(int N, double L, double lDeb, int k, double* bound);
static double far_radius_l(int N, double L, double lDeb, int k, int level, double* bound, bool cutterm = true);
static bool form_measured(const mdqt_ctx* s);
static double tier_radius(const mdqt_ctx* s, int k, int level, double* bound);
static void tier_radii(const mdqt_ctx* s, N3BArgs& a);
static double error_eps(const mdqt_ctx* s, const N3BArgs& a);
extern "C" double mdqt_get_const(const mdqt_ctx* s, const char* n) {
    if (!strcmp(n, "gamToEinsteinFreq")) return s->gamToE;
    if (!strcmp(n, "quantumTimestep")) return s->dtQ;
    if (!strcmp(n, "plasmaToQuantumTimestepRatio")) return s->ratio;
    if (!strcmp(n, "plasVelToQuantVel")) return s->pv2q;
    if (!strcmp(n, "vKick")) return s->vKick;
    if (!strcmp(n, "vKickDP")) return s->vKickDP;
    if (!strcmp(n, "lDeb")) return s->lDeb;
    if (!strcmp(n, "L")) return s->L;
    if (!strcmp(n, "decayRatioD5Halves")) return s->r;
    if (!strcmp(n, "kRat")) return s->kRat;
    if (!strcmp(n, "force_segments")) return s->nseg;
    if (!strcmp(n, "force_scheme")) return s->use_n3b ? 3 : s->use_n3 ? 2 : 1;
    if (!strcmp(n, "force_sort")) return s->use_n3b ? s->sort_mode : 0;
    if (!strcmp(n, "force_ax1")) return s->ax1_mode;
    if (!strcmp(n, "force_reduce_mask")) return s->tmask_mode;
    if (!strcmp(n, "force_tile_split")) return s->split_opt;
    if (!strcmp(n, "force_split_cus")) return s->split_cus;
    if (!strcmp(n, "force_tile_split_pairs")) return s->nsplit;
    if (!strcmp(n, "device_cus")) {                    // compute units of the context's device
        int ncu = 0;
        return hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, s->dev) == hipSuccess ? ncu : -1;
    }
    if (!strcmp(n, "force_balance")) return s->balance_opt;
    if (!strcmp(n, "force_balance_ratio")) return s->balance_ratio;           // max / mean rank work (NaN: not sharded yet)
    if (!strcmp(n, "force_balance_ratio_equal")) return s->balance_ratio_eq;  // the same for equal block counts
    if (!strcmp(n, "n3b_block_lo")) return s->use_n3b ? s->n3b.Plo : 0;
    if (!strcmp(n, "n3b_block_hi")) return s->use_n3b ? s->n3b.Phi : 0;
    if (!strcmp(n, "force_skip_radius") || !strcmp(n, "force_tail_bound")) {   // the tile-pair skip radius
        double bound;                                  // and its force bound (0: exact, r = L/2)
        const double r = (s->use_n3b && s->sort_mode == 1) ? skip_radius(s, &bound) : (bound = 0., s->L / 2.);
        if (n[6] == 's') return r;
        N3BArgs ea{};                                  // (what the call's sums hold: error_eps > 0)
        ea.Rcut = s->L / 2.; ea.Rskip = r;
        if (s->use_n3b) tier_radii(s, ea);
        if (s->use_n3b && (tail_measured(s) || form_measured(s)) && error_eps(s, ea) > 0.) {
            // mode 1: the running maximum of the per-tile sums each call met after the exact pass
            // (1e-12 relative: the device sum's rounding); NaN until a force call has measured.  With
            // force_form_mode 1 the sums hold the error-bounded forms' terms too: the bound on every
            // ion's total deviation from the exact sum to L/2 (held to force_error_eps)
            unsigned long long h[8];
            if (!s->dTailSt || hipStreamSynchronize(s->stream) != hipSuccess ||
                hipMemcpy(h, s->dTailSt, sizeof h, hipMemcpyDeviceToHost) != hipSuccess || h[4] == 0) return NAN;
            return u64_as_double(h[0]) * (1. + 1e-12);
        }
        return bound;
    }
    // mode 1 diagnostics: the largest per-tile sum the skip radius alone left (before the exact
    // pass), the tiles that exceeded eps so far, the measured force calls, the model scale
    if (!strcmp(n, "force_tail_raw_bound") || !strcmp(n, "force_tail_fixed_tiles") ||
        !strcmp(n, "force_tail_calls")) {
        unsigned long long h[8] = {0, 0, 0, 0, 0, 0, 0, 0};
        if (s->dTailSt && (hipStreamSynchronize(s->stream) != hipSuccess ||
                           hipMemcpy(h, s->dTailSt, sizeof h, hipMemcpyDeviceToHost) != hipSuccess)) return NAN;
        if (n[11] == 'r') return u64_as_double(h[1]) * (1. + 1e-12);
        return (double)(n[11] == 'f' ? h[2] : h[4]);
    }
    if (!strcmp(n, "force_tail_scale")) return s->tail_scale;
    if (!strcmp(n, "force_tail_model_bound")) {       // mode 1: the model bound r_t was chosen by
        double bound;
        const double r = (s->use_n3b && tail_measured(s)) ? tail_radius_sum(s, &bound) : (bound = 0., 0.);
        (void)r;
        return bound;
    }
    if (!strcmp(n, "force_tail_mode")) return s->tail_mode;
    if (!strcmp(n, "force_form_mode")) return s->form_mode;
    if (!strcmp(n, "force_form_measured")) return form_measured(s) ? 1. : 0.;
    if (!strcmp(n, "force_error_eps")) {               // the eps the measured sums are held to (0: none)
        if (!(s->use_n3b && (tail_measured(s) || form_measured(s)))) return 0.;
        N3BArgs a{};
        double b;
        a.Rcut = s->L / 2.;
        a.Rskip = skip_radius(s, &b);
        tier_radii(s, a);
        return error_eps(s, a);
    }
    if (!strcmp(n, "force_far_radius") || !strcmp(n, "force_far_bound")) {   // the far pair form's radius
        double bound;                                  // and force bound (0: off, r = L/2)
        const double r = (s->use_n3b && s->sort_mode != 0 && s->force_variant == 1 && !s->guard)
                             ? tier_radius(s, s->far_exp, 1, &bound) : (bound = 0., s->L / 2.);
        return n[10] == 'r' ? r : bound;
    }
    if (!strcmp(n, "force_mid_radius") || !strcmp(n, "force_mid_bound")) {   // the mid form's radius
        double bound;                                  // and force bound (0: off, r = L/2)
        const double r = (MDQT_EXP_TAB && s->use_n3b && s->sort_mode != 0 && s->force_variant == 1 && !s->guard)
                             ? tier_radius(s, s->mid_exp, 5, &bound) : (bound = 0., s->L / 2.);
        return n[10] == 'r' ? r : bound;
    }
    if (!strcmp(n, "force_ufar_radius") || !strcmp(n, "force_ufar_bound")) {   // the ultra-far form's
        double bound;                                  // radius and force bound (0: off, r = L/2)
        double r = (s->use_n3b && s->sort_mode != 0 && s->force_variant == 1 && !s->guard)
                       ? tier_radius(s, s->ufar_exp, 3, &bound) : (bound = 0., s->L / 2.);
        if (r < s->L / 2. && s->L / 2. > 80. * s->lDeb) { r = s->L / 2.; bound = 0.; }
        double b32 = 0.;                               // + the f32 shell beyond force_ufar32_radius
        if (r < s->L / 2. && MDQT_UFAR32) tier_radius(s, s->ufar_exp, 4, &b32);
        return n[11] == 'r' ? r : bound + b32;
    }
    if (!strcmp(n, "force_ufar32_radius")) {          // the f32 ultra-far form's radius (L/2: off)
        double bound;
        const double r3 = mdqt_get_const(s, "force_ufar_radius");
        return (r3 < s->L / 2. && MDQT_UFAR32) ? tier_radius(s, s->ufar_exp, 4, &bound) : s->L / 2.;
    }
    if (!strcmp(n, "force_vfar_radius") || !strcmp(n, "force_vfar_bound")) {   // the very-far form's
        double bound;                                  // radius and force bound (0: off, r = L/2)
        const double r = (s->use_n3b && s->sort_mode != 0 && s->force_variant == 1 && !s->guard)
                             ? tier_radius(s, s->vfar_exp, 2, &bound) : (bound = 0., s->L / 2.);
        return n[11] == 'r' ? r : bound;
    }
    if (!strcmp(n, "fused_step")) return s->fused_opt;
    if (!strcmp(n, "qt_im01")) return s->qc.im01;
    if (!strcmp(n, "potential_n3")) return s->n3_potential;
    if (!strcmp(n, "potential_plan")) return s->pot_plan;
    if (!strcmp(n, "force_n3b_pairs")) return s->n3b_pairs;
    if (!strcmp(n, "md_step_fused")) return s->last_fused;     // 1: the last MD step was one k_md_step launch
    if (!strcmp(n, "qt_kernel")) return s->last_qt_kernel;     // instance of the last substep launch (QTKernel)
    if (!strcmp(n, "qt_kernel_nseg")) return s->last_qt_nseg;  // force partials its prologue summed
    if (!strcmp(n, "force_slots")) return s->nslots;           // Newton-3 tile slots (0: other schemes)
    if (!strcmp(n, "n3b_blocks")) return s->use_n3b ? s->n3b.Phi - s->n3b.Plo : 0;   // this rank's blocks
    if (!strcmp(n, "n3b_block_count")) return s->use_n3b ? s->n3b.NB : 0;             // all blocks
    if (!strcmp(n, "slab_S")) return s->S;
    if (!strncmp(n, "gs", 2)) return s->gs[atoi(n + 2)];
    return NAN;
}

// ---------------------------------------------------------------------------------------------
// state transfer (host <-> HBM); psi: host [N][12][2] interleaved <-> device [24][S]
// ---------------------------------------------------------------------------------------------

static int upload(mdqt_ctx* s, const double* R, const double* V, size_t ld, const double* psi,
                  const double* tPart) {
    const int N = s->N, S = s->S, W = s->p.world_size;
    HIPCHK(hipSetDevice(s->dev));
    if (R) {
        std::vector<double> h((size_t)3 * S * W, 0.);
        for (int g = 0; g < N; ++g) {
            const int w = g / S, l = g - w * S;
            for (int c = 0; c < 3; ++c) h[(size_t)w * 3 * S + (size_t)c * S + l] = R[(size_t)c * ld + g];
        }
        HIPCHK(hipMemcpyAsync(s->dR, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice, s->stream));
        int oor = 0;                                     // positions outside [-L/8, 9L/8]?
        const double plo = -0.125 * s->L, phi = 1.125 * s->L;
        for (size_t k = 0; k < (size_t)3 * N && !oor; ++k) {
            const double x = R[(k / N) * ld + k % N];
            if (!(x >= plo && x <= phi)) oor = 1;
        }
        s->guard = oor != 0;
        const int zero = 0;
        HIPCHK(hipMemcpyAsync(s->dFlags, &zero, sizeof zero, hipMemcpyHostToDevice, s->stream));
        HIPCHK(hipStreamSynchronize(s->stream));
    }
    const int lo = s->lo, n = s->nloc;
    if (V) {
        std::vector<double> h((size_t)3 * S, 0.);
        for (int c = 0; c < 3; ++c)
            for (int i = 0; i < n; ++i) h[(size_t)c * S + i] = V[(size_t)c * ld + lo + i];
        HIPCHK(hipMemcpyAsync(s->dV, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice, s->stream));
        HIPCHK(hipStreamSynchronize(s->stream));
    }
    if (psi) {
        std::vector<double> h((size_t)24 * S, 0.);
        for (int i = 0; i < n; ++i)
            for (int k = 0; k < 24; ++k) h[(size_t)k * S + i] = psi[(size_t)(lo + i) * 24 + k];
        HIPCHK(hipMemcpyAsync(s->dPsi, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice, s->stream));
        HIPCHK(hipStreamSynchronize(s->stream));
    }
    if (tPart) {
        std::vector<double> h((size_t)S, 0.);
        for (int i = 0; i < n; ++i) h[i] = tPart[lo + i];
        HIPCHK(hipMemcpyAsync(s->dTp, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice, s->stream));
        HIPCHK(hipStreamSynchronize(s->stream));
    }
    return 0;
}

extern "C" int mdqt_set_state(mdqt_ctx* s, int N, const double* R, const double* V, size_t ld,
                              const double* psi, const double* tPart, double t) {
    if (!s) return fail("NULL context");
    if (settle_forces(s)) return -1;                   // pending partials of the previous positions
    const bool sameN = N == s->N;
    if (!sameN && resize(s, N)) return -1;
    if (ld < (size_t)N) return fail("ld < N");
    if (upload(s, R, V, ld, psi, tPart)) return -1;
    if (R && tail_reset(s, sameN)) return -1;          // new positions: the tail statistics restart
    s->t = t;
    return 0;
}

extern "C" int mdqt_set_forces(mdqt_ctx* s, const double* F, size_t ld) {
    s->f_pending = false;
    s->rs_pending = false;
    const int S = s->S, lo = s->lo, n = s->nloc;
    std::vector<double> h((size_t)3 * S, 0.);
    for (int c = 0; c < 3; ++c)
        for (int i = 0; i < n; ++i) h[(size_t)c * S + i] = F[(size_t)c * ld + lo + i];
    HIPCHK(hipSetDevice(s->dev));
    HIPCHK(hipMemcpyAsync(s->dF, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    return 0;
}

extern "C" int mdqt_get_state(mdqt_ctx* s, double* R, double* V, double* F, size_t ld, double* psi,
                              double* tPart, double* t) {
    if (!s) return fail("NULL context");
    const int N = s->N, S = s->S, W = s->p.world_size, lo = s->lo, n = s->nloc;
    if (ld < (size_t)N) return fail("ld < N");
    HIPCHK(hipSetDevice(s->dev));
    if (check_range_flag(s)) return -1;
    if (F && settle_forces(s)) return -1;
    if (R) {
        std::vector<double> h((size_t)3 * S * W);
        HIPCHK(hipMemcpyAsync(h.data(), s->dR, h.size() * sizeof(double), hipMemcpyDeviceToHost, s->stream));
        HIPCHK(hipStreamSynchronize(s->stream));
        for (int g = 0; g < N; ++g) {
            const int w = g / S, l = g - w * S;
            for (int c = 0; c < 3; ++c) R[(size_t)c * ld + g] = h[(size_t)w * 3 * S + (size_t)c * S + l];
        }
    }
    auto get3 = [&](const double* d, double* out) -> int {
        std::vector<double> h((size_t)3 * S);
        HIPCHK(hipMemcpyAsync(h.data(), d, h.size() * sizeof(double), hipMemcpyDeviceToHost, s->stream));
        HIPCHK(hipStreamSynchronize(s->stream));
        for (int c = 0; c < 3; ++c)
            for (int i = 0; i < n; ++i) out[(size_t)c * ld + lo + i] = h[(size_t)c * S + i];
        return 0;
    };
    if (V && get3(s->dV, V)) return -1;
    if (F && get3(s->dF, F)) return -1;
    if (psi) {
        std::vector<double> h((size_t)24 * S);
        HIPCHK(hipMemcpyAsync(h.data(), s->dPsi, h.size() * sizeof(double), hipMemcpyDeviceToHost, s->stream));
        HIPCHK(hipStreamSynchronize(s->stream));
        for (int i = 0; i < n; ++i)
            for (int k = 0; k < 24; ++k) psi[(size_t)(lo + i) * 24 + k] = h[(size_t)k * S + i];
    }
    if (tPart) {
        std::vector<double> h((size_t)S);
        HIPCHK(hipMemcpyAsync(h.data(), s->dTp, h.size() * sizeof(double), hipMemcpyDeviceToHost, s->stream));
        HIPCHK(hipStreamSynchronize(s->stream));
        for (int i = 0; i < n; ++i) tPart[lo + i] = h[i];
    }
    if (t) *t = s->t;
    return 0;
}

extern "C" int mdqt_get_N(const mdqt_ctx* s) { return s ? s->N : -1; }
extern "C" double mdqt_get_time(const mdqt_ctx* s) { return s->t; }
extern "C" int mdqt_set_time(mdqt_ctx* s, double t) { s->t = t; return 0; }
extern "C" uint64_t mdqt_get_qstep_index(const mdqt_ctx* s) { return s->qidx; }
extern "C" int mdqt_set_qstep_index(mdqt_ctx* s, uint64_t q) { s->qidx = q; return 0; }
extern "C" int mdqt_get_counters(const mdqt_ctx* s, int* c0, unsigned* counter, double* Epot, double* Epot0) {
    if (c0) *c0 = s->c0;
    if (counter) *counter = s->counter;
    if (Epot) *Epot = s->Epot;
    if (Epot0) *Epot0 = s->Epot0;
    return 0;
}

// ---------------------------------------------------------------------------------------------
// init (SpeedUp:289-348): drand48 rejection sampling, bit-exact with the reference stream
// ---------------------------------------------------------------------------------------------

// ---------------------------------------------------------------------------------------------
// init() (SpeedUp:289-348): rejection sampling of N9L candidate triples from ONE drand48 stream;
// a kept triple consumes 4 more draws for its wavefunction.
//
// Sequentially that is 3 N9L + 4 N draws (2.2e9 at N0 = 1M: ~13 s on one core).  In parallel,
// with the same stream and the same result bit for bit: a candidate starting at draw index p is
// kept iff ok(u_p) && ok(u_p+1) && ok(u_p+2), independently of the walk, so (1) threads scan
// disjoint ranges of draw indices (LCG jump-ahead to each range start) and list every p that
// WOULD be kept (rate 1/729); (2) one pass walks the candidates: from p the walk visits p, p+3,
// ... until the first listed p' in the same residue class mod 3, takes it and continues at
// p' + 7 (so the class shifts by one per kept ion), counting candidates up to N9L; (3) the kept
// ions' 7 draws are regenerated by jump-ahead, in parallel.  If the walk runs past the scanned
// range (more ions than the bound allows) it finishes sequentially from there.
// ---------------------------------------------------------------------------------------------

extern "C" int mdqt_init(mdqt_ctx* s) {
    if (!s) return fail("NULL context");
    const double L = s->L;
    const double N9L = (unsigned)(9. * 9. * 9. * (L * L * L) * 3. / (4. * M_PI));   // :299
    int threads = s->init_threads;
    if (threads <= 0) {
        const unsigned hc = std::thread::hardware_concurrency();
        threads = (int)std::min(16u, hc ? hc : 1u);
    }
    const long Nbound = (long)s->p.N0 + 1000 + (long)(20. * sqrt((double)s->p.N0 + 1.));
    uint64_t xend = 0;
    const std::vector<InitIon> ions =
        init_sample(srand48_state(s->p.seed), L, (long)N9L, Nbound, threads, &xend);   // :1219, :303-335
    s->x48 = xend;
    std::vector<double> X, Y, Z, psi((size_t)24 * ions.size(), 0.);
    for (size_t k = 0; k < ions.size(); ++k) {
        X.push_back(ions[k].x); Y.push_back(ions[k].y); Z.push_back(ions[k].z);
        psi[24 * k] = ions[k].w0; psi[24 * k + 2] = ions[k].w2; psi[24 * k + 3] = ions[k].w3;
    }
    const int N = (int)X.size();
    std::vector<double> R((size_t)3 * N), V((size_t)3 * N, 0.), tp((size_t)N, 0.);
    for (int i = 0; i < N; ++i) { R[i] = X[i]; R[(size_t)N + i] = Y[i]; R[(size_t)2 * N + i] = Z[i]; }
    if (resize(s, N)) return -1;
    if (upload(s, R.data(), V.data(), N, psi.data(), tp.data())) return -1;
    if (tail_reset(s)) return -1;
    if (s->dX48) {                                   // the qstep draws continue this stream
        unsigned long long x = s->x48;
        HIPCHK(hipMemcpy(s->dX48, &x, sizeof x, hipMemcpyHostToDevice));
    }
    double e;
    if (mdqt_epotential(s, &e)) return -1;                                           // :345-347
    s->Epot0 = s->Epot;
    s->c0 = -1;
    s->t = 0.;
    s->qidx = 0;
    return 0;
}

// ---------------------------------------------------------------------------------------------
// hot path
// ---------------------------------------------------------------------------------------------

// smallest d with fl(d / L) >= 0.5 in IEEE double (the device's division is IEEE too), so that
// round(dx/L) == (dx >= T) - (dx <= -T) for |dx| < 1.25 L: the minimum image without a division
static double mic_threshold(double L) {
    double d = 0.5 * L;
    while (d > 0 && d / L >= 0.5) d = nextafter(d, 0.);
    while (d / L < 0.5) d = nextafter(d, INFINITY);
    return d;
}

static void fill_pair_consts(ForceArgs& a, double L, double lDeb, int variant) {
    a.L = L; a.lDeb = lDeb; a.Rcut = L / 2.;               // :196
    a.invlDeb = 1. / lDeb;                                  // :224
    a.micT = mic_threshold(L);
    a.micGuard = 1.25 * L;
    a.variant = variant;
}

static ForceArgs force_args(mdqt_ctx* s, double* out);

// The error-bounded tail radius: the smallest r in (0, L/2] with (N - 1) g(r) <= eps, where
// g(r) = (1/r + 1/lDeb) exp(-r/lDeb) / r is |F| of one pair at distance r (SpeedUp:224 times r),
// decreasing in r.  A skipped tile pair's boxes are >= r_t apart, so each of its pairs is, and the
// pairs an ion loses number at most N - 1: |dF_i| <= (N - 1) g(r_t) <= eps (rigorous; the actual
// tail is far smaller — its terms have random directions).  L/2 (exact: nothing extra skipped)
// when eps = 0 or (N - 1) g(L/2) > eps.  bound = (N - 1) g(r_t) (0 when exact).
static double tail_g(double r, double lDeb) { return (1. / r + 1. / lDeb) * exp(-r / lDeb) / r; }
static double tail_radius(int N, double L, double lDeb, int k, double* bound) {
    const double Rcut = L / 2.;
    *bound = 0.;
    if (k <= 0 || N < 2) return Rcut;
    const double eps = pow(10., -k);
    const double n1 = (double)(N - 1);
    if (n1 * tail_g(Rcut, lDeb) > eps) return Rcut;
    double lo = 0., hi = Rcut;                      // n1 g(hi) <= eps < n1 g(lo)
    for (int it = 0; it < 200 && hi - lo > 1e-12 * Rcut; ++it) {
        const double m = 0.5 * (lo + hi);
        if (m > 0 && n1 * tail_g(m, lDeb) <= eps) hi = m; else lo = m;
    }
    *bound = n1 * tail_g(hi, lDeb);
    return hi;
}
// force_tail_mode 1: r_t from a model of the bound the device measures, per 16-ion sub-tile a sum over
// the dropped sub-blocks (a, b) of n_b g(sub-box gap): at density rho = N / L^3 the sub-tiles with box
// gap in [x, x + dx] hold about rho 4 pi (x + delta)^2 dx ions, delta = two sub-tile widths
// (16 / rho)^(1/3) bounding the box extents, so B(r) = rho int_r^(L/2) 4 pi (x + delta)^2 g(x) dx
// (beyond L/2 only pairs beyond the cutoff); r_t the smallest r with m s B(r) <= eps (m = kTailMargin, a
// margin for the model, s = tail_scale: 1, raised by tail_check when a configuration's measured
// sums exceeded eps), never beyond the a-priori radius (rigorous for any configuration).  The
// model only picks r_t: the kernel measures every tile's sum and k_tail_fix enforces eps.
// Memoised per context.
static double tail_model(double r, int N, double L, double lDeb) {
    const double rho = N / (L * L * L), delta = 2. * cbrt(16. / rho), hi = L / 2.;
    if (r >= hi) return 0.;
    const int n = 2000;                             // Simpson on [r, L/2]
    const double h = (hi - r) / n;
    auto f = [&](double x) { return 4. * M_PI * (x + delta) * (x + delta) * tail_g(x, lDeb); };
    double acc = f(r) + f(hi);
    for (int i = 1; i < n; ++i) acc += (i & 1 ? 4. : 2.) * f(r + i * h);
    return rho * acc * h / 3.;
}
// the model's margin: the measured per-sub-tile sums stayed at ~0.7 of the model at N = 1e6 (C4 and
// C2's parameters, uniform init()), and the exact pass enforces eps whenever a configuration exceeds
// it, so the margin only sets how rarely that pass runs
constexpr double kTailMargin = 1.25;
static double tail_radius_sum(const mdqt_ctx* s, double* bound) {
    const int N = s->N, k = s->tail_exp;
    const double L = s->L, lDeb = s->lDeb, Rcut = L / 2.;
    *bound = 0.;
    if (k <= 0 || N < 2) return Rcut;
    const double sc = s->tail_scale;
    if (s->tail_key[0] == N && s->tail_key[1] == L && s->tail_key[2] == lDeb && s->tail_key[3] == k &&
        s->tail_key[4] == sc) {
        *bound = s->tail_val[1];
        return s->tail_val[0];
    }
    const double eps = pow(10., -k);
    double r = Rcut, b = 0.;
    // only where the a-priori radius is below L/2 (N ~ 1e6): elsewhere the model would skip a sliver
    // just inside L/2 for nothing, and those sizes keep the exact cutoff
    double b0;
    const double ra = tail_radius(N, L, lDeb, k, &b0);
    if (ra < Rcut) {
        double lo = 0., hi = Rcut;
        for (int it = 0; it < 60 && hi - lo > 1e-9 * Rcut; ++it) {
            const double m = 0.5 * (lo + hi);
            if (m > 0 && kTailMargin * sc * tail_model(m, N, L, lDeb) <= eps) hi = m; else lo = m;
        }
        r = hi;
        b = tail_model(hi, N, L, lDeb);
        if (r > ra) { r = ra; b = b0; }              // the a-priori radius bounds any configuration
    }
    s->tail_key[0] = N; s->tail_key[1] = L; s->tail_key[2] = lDeb; s->tail_key[3] = k; s->tail_key[4] = sc;
    s->tail_val[0] = r; s->tail_val[1] = b;
    *bound = b;
    return r;
}
// the context's skip radius: mode 1 (measured and enforced) in spatial order at every world size
// (the per-tile sums are all-reduced, so 1 and W ranks run the same algorithm), else a priori
// — for the fast pair form only: k_tail_fix recomputes the listed tiles in that form (pair_ft<1>, the
// cutoff on dr < Rcut), so the other variants keep the a-priori radius
static bool tail_measured(const mdqt_ctx* s) { return s->tail_mode == 1 && s->sort_mode == 1 && s->force_variant == 1; }
static double skip_radius(const mdqt_ctx* s, double* bound) {
    return tail_measured(s) ? tail_radius_sum(s, bound) : tail_radius(s->N, s->L, s->lDeb, s->tail_exp, bound);
}
// force_tail_mode 1 at a host synchronisation point: if tiles exceeded eps since the last check
// (k_tail_fix summed their skipped tile pairs exactly, so those calls met eps anyway), the density
// model underestimated this configuration's tail by u = (largest measured sum) / (the model's at
// r_t): the next calls take r_t for tail_scale = max(2 tail_scale, 2^ceil(log2 u)) — capped at the
// a-priori radius — and stderr says so.  Every rank sees the same all-reduced sums, so ranks
// widen alike.
static double model_total(const mdqt_ctx* s);
static int tail_check(mdqt_ctx* s) {
    if (!s->dTailSt || !s->use_n3b || !(tail_measured(s) || form_measured(s))) return 0;
    unsigned long long h[8];
    HIPCHK(hipMemcpyAsync(h, s->dTailSt, sizeof h, hipMemcpyDeviceToHost, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    if (h[2] <= s->tail_seen) return 0;
    double b0, b1;
    const double r0 = tail_radius_sum(s, &b0);
    const double raw = u64_as_double(h[1]);
    b0 = model_total(s);                            // (the tail's model bound + the tiers', force_form_mode 1)
    const double u = b0 > 0. ? raw / b0 : INFINITY;
    // a power of two: the sums' last bits (atomic order, the ranks' partial sums) cannot move it
    s->tail_scale = std::max(2. * s->tail_scale, std::isfinite(u) && u < 1e300 ? exp2(ceil(log2(u))) : 1e300);
    const double r1 = tail_radius_sum(s, &b1);
    if (s->tail_warned++ < 8)                       // (rate-limited: a few lines per context)
        fprintf(stderr, "mdqt: force error bound exceeded on %llu tile(s) so far (largest per-tile sum %.3e; the model's "
                "%.3e at r_t = %.4f): corrected by the exact pass; r_t widened to %.4f (the tiers' radii likewise)\n",
                (unsigned long long)h[2], raw, b0, r0, r1);
    s->tail_seen = h[2];
    return 0;
}

// the enforcement after a force call's tail sums are complete: list the tiles over eps, add their
// skipped pairs exactly (k_tail_fix) to `out` (F, or this rank's dense partial)
static int tail_enforce(mdqt_ctx* s, const N3BArgs& a, double* out) {
    const double eps = error_eps(s, a);
    HIPCHK(launch_tail_max(a.tailb, a.T, eps, s->dTailSt, s->dTailList, s->stream));
    HIPCHK(launch_tail_fix(a, s->dTailSt, s->dTailList, out, s->stream));
    return 0;
}

// in-process rank group: the ranks' per-tile sums summed in rank order and handed to every rank,
// which then enforces on its own dense partial — the ncclAllReduce of a real group (mdqt_forces)
static int local_tail(mdqt_ctx* s) {
    bool any = false;
    for (mdqt_ctx* q : s->local) any = any || q->tail_pending;
    if (!any) return 0;
    const int T = s->tail_args.T, T4 = 4 * T;                 // per-sub-tile sums
    std::vector<double> sum((size_t)T4, 0.), h((size_t)T4);
    for (mdqt_ctx* q : s->local) {
        if (!q->tail_pending || q->tail_args.T != T) return fail("local group: rank %d has no tail sums", q->p.rank);
        HIPCHK(hipSetDevice(q->dev));
        HIPCHK(hipMemcpyAsync(h.data(), q->tail_args.tailb, (size_t)T4 * sizeof(double), hipMemcpyDeviceToHost, q->stream));
        HIPCHK(hipStreamSynchronize(q->stream));
        for (int t = 0; t < T4; ++t) sum[t] = sum[t] + h[t];
    }
    for (mdqt_ctx* q : s->local) {
        HIPCHK(hipSetDevice(q->dev));
        HIPCHK(hipMemcpyAsync(q->tail_args.tailb, sum.data(), (size_t)T4 * sizeof(double), hipMemcpyHostToDevice, q->stream));
        if (tail_enforce(q, q->tail_args, q->dFr)) return -1;
        HIPCHK(hipStreamSynchronize(q->stream));
        q->tail_pending = false;
    }
    for (mdqt_ctx* q : s->local) {                 // every rank reacts here, at the same point
        HIPCHK(hipSetDevice(q->dev));
        if (tail_check(q)) return -1;
    }
    HIPCHK(hipSetDevice(s->dev));
    return 0;
}

// the far radii: the smallest r with (N - 1) g(r) err(r) <= 10^-k, err the relative error of a term
// at distance r in the form (far: kFarRelErr; very far: (r/lDeb + 3) kRsqRawErr + kExp5RelErr) —
// L/2 (= never) and bound 0 when k = 0 or that r is >= L/2; bound = (N - 1) g(r) err(r)
static double far_err(double r, double lDeb, int level) {
    if (level == 5) return (r / lDeb + 3.) * (kRsq1RelErr + 0x1p-52) + kTab4RelErr;   // the mid form
    if (level == 4) return (r / lDeb) * kUfar32A + kUfar32B;   // the f32 ultra-far form (MDQT_UFAR32)
    if (level == 3) return (r / lDeb) * (kRsqRawErr + 0x1p-24) + 3. * kRsqRawErr + kExp2fRelErr;
    return level == 2 ? (r / lDeb + 3.) * kRsqRawErr + kExp5RelErr : kFarRelErr;
}
static double far_radius_l(int N, double L, double lDeb, int k, int level, double* bound, bool cutterm) {
    const double Rcut = L / 2.;
    *bound = 0.;
    if (k <= 0 || N < 2) return Rcut;
    const double eps = pow(10., -k), n1 = (double)(N - 1);
    // level 4 (f32) decides the cutoff on its f32 r^2 (relative error <= 6 2^-24): pairs within
    // 3 2^-24 Rcut of L/2 may land on either side, each at most g(Rcut (1 - 2^-20)) — a constant term
    // (not with force_form_mode 1, cutterm false: the plan keeps the f32 form off the cutoff)
    const double cut = level == 4 && cutterm ? n1 * tail_g(Rcut * (1. - 0x1p-20), lDeb) : 0.;
    auto b = [&](double r) { return n1 * tail_g(r, lDeb) * far_err(r, lDeb, level) + cut; };
    if (b(Rcut) > eps) return Rcut;
    double lo = 0., hi = Rcut;
    for (int it = 0; it < 200 && hi - lo > 1e-12 * Rcut; ++it) {
        const double m = 0.5 * (lo + hi);
        if (m > 0 && b(m) <= eps) hi = m; else lo = m;
    }
    *bound = b(hi);
    return hi;
}
static double far_radius(int N, double L, double lDeb, int k, double* bound) {
    return far_radius_l(N, L, lDeb, k, 1, bound);
}

// force_form_mode 1 (round 6): the tiers' radii from a density model of the per-sub-tile form sums the
// plan measures (k_n3b_plan), as tail_model for the tail: at density rho the sub-tiles with box gap in
// [x, x + dx] hold about rho 4 pi (x + delta)^2 dx ions, so a sub-tile's sum over a tier's sub-blocks (gap
// >= r) is about F(r) = rho int_r^hi 4 pi (x + delta)^2 g(x) err(x) dx, hi = r_t (nothing beyond it is
// evaluated).  The radius is the smallest r with m s F(r) <= 10^-k (m = kTailMargin, s = tail_scale:
// raised with r_t's when a call's sums exceeded its eps), never beyond the a-priori radius (rigorous for
// any configuration; level 4 without the cutoff term).  The model only picks the radii: the plan measures
// every tile's sum and k_tail_fix enforces the call's eps (error_eps).
// (force_sort 1 and 2 alike: 2 runs the same plan without skipping, and must give the same forms)
static bool form_measured(const mdqt_ctx* s) {
    return s->form_mode >= 1 && s->use_n3b && s->tail_mode == 1 && s->sort_mode >= 1 && s->force_variant == 1 &&
           !s->guard;
}
// a tier's eps (k > 0): 10^-k, + (force_form_mode 2, where the tail skips nothing: r_t = L/2) an equal
// share of the tail's 10^-tail_exp among the tiers with k > 0 — the per-ion total stays 10^-tail_exp + sum
// 10^-k, as where the tail is active
static double tier_eps(const mdqt_ctx* s, int k) {
    if (k <= 0) return 0.;
    double e = pow(10., -k);
    double tb;
    if (s->form_mode == 2 && form_measured(s) && s->tail_exp > 0 && tail_radius_sum(s, &tb) >= s->L / 2.) {
        const int n = (MDQT_EXP_TAB && s->mid_exp > 0) + (s->far_exp > 0) + (s->vfar_exp > 0) +
                      (s->ufar_exp > 0) * (MDQT_UFAR32 ? 2 : 1);
        e += pow(10., -s->tail_exp) / n;
    }
    return e;
}
static double form_model(double r, double hi, int N, double L, double lDeb, int level) {
    const double rho = N / (L * L * L), delta = 2. * cbrt(16. / rho);
    if (r >= hi) return 0.;
    const int n = 2000;                             // Simpson on [r, hi]
    const double h = (hi - r) / n;
    auto f = [&](double x) { return 4. * M_PI * (x + delta) * (x + delta) * tail_g(x, lDeb) * far_err(x, lDeb, level); };
    double acc = f(r) + f(hi);
    for (int i = 1; i < n; ++i) acc += (i & 1 ? 4. : 2.) * f(r + i * h);
    return rho * acc * h / 3.;
}
// the model radius of a tier (context-free; mdqt_tier_radius_model exports it for the CPU tests): the
// smallest r with m s F(r) <= eps (10^-k, or tier_eps) on [0, hi], hi = r_t, capped by the a-priori
// radius of 10^-k (its bound <= 10^-k <= eps); L/2 = off
static double model_tier_radius(int N, double L, double lDeb, int k, double eps, int level, double hi, double sc,
                                double* bound) {
    const double Rcut = L / 2.;
    *bound = 0.;
    if (k <= 0 || N < 2) return Rcut;
    double ba;
    const double ra = far_radius_l(N, L, lDeb, k, level, &ba, false);
    double lo = 0., up = hi;
    for (int it = 0; it < 60 && up - lo > 1e-9 * Rcut; ++it) {
        const double m = 0.5 * (lo + up);
        if (m > 0 && kTailMargin * sc * form_model(m, hi, N, L, lDeb, level) <= eps) up = m; else lo = m;
    }
    double r = up, b = form_model(up, hi, N, L, lDeb, level);
    if (r >= ra) { r = ra; b = ba; }                // the a-priori radius bounds any configuration
    if (r >= hi) { r = Rcut; b = 0.; }              // (nothing evaluated that far: the tier is off)
    *bound = b;
    return r;
}
// a tier's radius (L/2: off) and bound: a priori (force_form_mode 0) or the model's (1; memoised per context)
static double tier_radius(const mdqt_ctx* s, int k, int level, double* bound) {
    if (!form_measured(s)) return far_radius_l(s->N, s->L, s->lDeb, k, level, bound);
    *bound = 0.;
    if (k <= 0 || s->N < 2) return s->L / 2.;
    const double sc = s->tail_scale, eps = tier_eps(s, k);
    double* key = s->form_key[level];
    if (key[0] == s->N && key[1] == s->L && key[2] == s->lDeb && key[3] == eps && key[4] == s->tail_exp &&
        key[5] == sc) {
        *bound = s->form_val[level][1];
        return s->form_val[level][0];
    }
    double tb;
    const double hi = tail_radius_sum(s, &tb);      // r_t (L/2 where the tail is exact)
    double b;
    const double r = model_tier_radius(s->N, s->L, s->lDeb, k, eps, level, hi, sc, &b);
    key[0] = s->N; key[1] = s->L; key[2] = s->lDeb; key[3] = eps; key[4] = s->tail_exp; key[5] = sc;
    s->form_val[level][0] = r; s->form_val[level][1] = b;
    *bound = b;
    return r;
}
// C ABI for the CPU tests (no device needed): a tier's model radius and bound for given parameters,
// level as far_err (1 far, 2 very far, 3 ultra far, 4 ultra far in f32, 5 mid); hi = the skip radius
// the integral ends at (L/2 without a tail); apriori 1: force_form_mode 0's a-priori radius instead, 2: the
// a-priori radius without the f32 tier's cutoff term (the cap the model radius takes)
extern "C" int mdqt_tier_radius_model(int N, double L, double lDeb, int k, int level, double hi, double scale,
                                      int apriori, double* radius, double* bound) {
    if (!radius || !bound || N < 1 || !(L > 0.) || !(lDeb > 0.) || level < 1 || level > 5 || !(hi > 0.) ||
        !(scale > 0.) || apriori < 0 || apriori > 2)
        return -1;
    *radius = apriori ? far_radius_l(N, L, lDeb, k, level, bound, apriori == 1)
                      : model_tier_radius(N, L, lDeb, k, pow(10., -k), level, std::min(hi, L / 2.), scale, bound);
    return 0;
}
// the model's per-sub-tile sum at the current radii — the tail's where r_t < L/2, + the tiers' evaluated
// inside r_t (force_form_mode 1) — that tail_check compares the measured sums with
static double model_total(const mdqt_ctx* s) {
    double b = 0., t;
    const double rt = tail_radius_sum(s, &t);
    if (rt < s->L / 2.) b += t;
    if (form_measured(s)) {
        if (MDQT_EXP_TAB && tier_radius(s, s->mid_exp, 5, &t) < rt) b += t;
        if (tier_radius(s, s->far_exp, 1, &t) < rt) b += t;
        if (tier_radius(s, s->vfar_exp, 2, &t) < rt) b += t;
        if (tier_radius(s, s->ufar_exp, 3, &t) < rt) b += t;
        if (MDQT_UFAR32 && tier_radius(s, s->ufar_exp, 4, &t) < rt) b += t;
    }
    return b;
}
// the eps a force call's per-sub-tile sums are held to (k_tail_max): the tail's where r_t < L/2, plus
// (force_form_mode >= 1) the eps of every tier evaluated inside r_t (tier_eps)
static double error_eps(const mdqt_ctx* s, const N3BArgs& a) {
    double e = a.Rskip < a.Rcut ? pow(10., -s->tail_exp) : 0.;
    if (a.formm) {
        if (MDQT_EXP_TAB && a.Rmid < a.Rskip) e += tier_eps(s, s->mid_exp);
        if (a.Rfar < a.Rskip) e += tier_eps(s, s->far_exp);
        if (a.Rvfar < a.Rskip) e += tier_eps(s, s->vfar_exp);
        if (a.Rufar < a.Rskip) e += tier_eps(s, s->ufar_exp);
        if (MDQT_UFAR32 && a.Rufar32 < a.Rskip) e += tier_eps(s, s->ufar_exp);
    }
    return e;
}

// the tiers' radii of a force call (a.Rcut set): a priori or from the model (force_form_mode 1)
static void tier_radii(const mdqt_ctx* s, N3BArgs& a) {
    double bound;
    a.Rmid = MDQT_EXP_TAB ? tier_radius(s, s->mid_exp, 5, &bound) : a.Rcut;
    a.Rfar = tier_radius(s, s->far_exp, 1, &bound);
    a.Rvfar = tier_radius(s, s->vfar_exp, 2, &bound);
    a.Rufar = tier_radius(s, s->ufar_exp, 3, &bound);
    a.Rufar32 = MDQT_UFAR32 ? tier_radius(s, s->ufar_exp, 4, &bound) : a.Rcut;
    a.formm = form_measured(s) ? 1 : 0;
    a.u32lim2 = (a.Rcut * (1. - 0x1p-20)) * (a.Rcut * (1. - 0x1p-20));
    // f32's normal range: 2^t for t >= -126 (r <= 126 lDeb ln2 = 87 lDeb); never beyond it
    if (a.Rufar < a.Rcut && a.Rcut > 80. * s->lDeb) a.Rufar = a.Rcut;
    if (a.Rufar >= a.Rcut) a.Rufar32 = a.Rcut;
}

// the block-pair kernels' arguments for the current positions: with force_sort, the Hilbert order,
// the sorted copy and the tile boxes are recomputed here (mdqt_sort.hip)
static int n3b_args(mdqt_ctx* s, N3BArgs& a) {
    a = s->n3b;
    ForceArgs c = force_args(s, nullptr);
    a.Rall = s->dR; a.slots = s->dSlots; a.S = s->S;
    a.L = c.L; a.lDeb = c.lDeb; a.Rcut = c.Rcut; a.invlDeb = c.invlDeb; a.micT = c.micT;
    a.micGuard = c.micGuard; a.guard = c.guard;
    a.use_sort = 0; a.Rs = nullptr; a.perm = nullptr; a.boxes = nullptr; a.subboxes = nullptr; a.plan = nullptr;
    a.tmask = nullptr; a.tmw = 0;
    a.ax1 = s->ax1_mode;
    a.pairs = s->n3b_pairs;
    double bound;
    a.Rskip = skip_radius(s, &bound);
    a.tailb = nullptr;
    tier_radii(s, a);
    a.rc2 = a.Rcut * a.Rcut;
    if (s->sort_mode) {                            // Hilbert order + tile boxes (mdqt_sort.hip)
        SortArgs o;
        o.Rall = s->dR; o.N = s->N; o.S = s->S; o.Npad = a.Npad; o.L = s->L;
        o.keys = s->dKeys; o.keys2 = s->dKeys + s->N; o.ion = s->dIon; o.perm = s->dIon + s->N;
        o.tmp = s->dSortTmp; o.tmp_bytes = s->sortTmpBytes; o.Rs = s->dRs; o.boxes = s->dBoxes;
        o.subboxes = s->dSubBoxes;
        HIPCHK(launch_spatial_order(o, s->stream));
        a.use_sort = s->sort_mode; a.Rs = s->dRs; a.perm = o.perm; a.boxes = s->dBoxes; a.subboxes = s->dSubBoxes;
        // the per-sub-tile sums: where the tail skips pairs, or (force_form_mode 1) a tier is evaluated
        const bool tiers = a.formm && (a.Rmid < a.Rskip || a.Rfar < a.Rskip || a.Rvfar < a.Rskip || a.Rufar < a.Rskip);
        if ((tail_measured(s) && a.Rskip < a.Rcut) || tiers) a.tailb = s->dTail;
        // the plan (k_n3b_plan): 256 tile-pair words per (P, db), then one J-step mask per (P, db)
        // and the per-J-tile masks of the block distances whose j-slots the block kernel writes (k_n3b_reduce
        // reads only those): T x ceil(nd / 64) words
        const size_t nplan = (size_t)std::max(a.Phi - a.Plo, 0) * a.nd * (kN3BBlock * kN3BBlock + 1);
        const int tmw = (a.nd + 63) / 64;
        const size_t need = nplan + (size_t)a.T * tmw;
        if (need > s->capPlan) {
            if (s->dPlan) HIPCHK(hipFree(s->dPlan));
            s->dPlan = nullptr;
            HIPCHK(hipMalloc((void**)&s->dPlan, need * sizeof(uint2)));
            s->capPlan = need;
        }
        a.plan = s->dPlan;
        // (no masks for a rank without blocks: nothing would clear or fill them — ADVICE r05)
        const bool masks = s->tmask_mode && a.Phi > a.Plo;
        a.tmw = masks ? tmw : 0;
        a.tmask = masks ? (unsigned long long*)(s->dPlan + nplan) : nullptr;
    }
    return 0;
}

static ForceArgs force_args(mdqt_ctx* s, double* out) {
    ForceArgs a;
    a.Rall = s->dR;
    a.Fpart = out;
    a.N = s->N; a.S = s->S;
    a.row_lo = s->lo; a.nrows = s->nloc;
    a.nseg = s->nseg; a.seglen = s->seglen;
    fill_pair_consts(a, s->L, s->lDeb, s->force_variant);
    a.guard = s->guard ? 1 : 0;
    return a;
}

// in-process rank group with block-pair Newton-3: F of this rank = the ranks' dense partials
// summed in rank order (RCCL's reduce-scatter in a real group).  Peers' force launches are
// complete: callers step the group in lockstep (all forces before any substeps).
static int local_reduce(mdqt_ctx* s) {
    if (!s->rs_pending) return 0;
    if (local_tail(s)) return -1;
    const int W = s->p.world_size;
    std::vector<const double*> h(W, nullptr);
    for (mdqt_ctx* q : s->local) {
        if (!q->dFr) return fail("local_reduce: rank %d has no partial forces", q->p.rank);
        h[q->p.rank] = q->dFr;
        HIPCHK(hipSetDevice(q->dev));
        HIPCHK(hipStreamSynchronize(q->stream));
    }
    HIPCHK(hipSetDevice(s->dev));
    if (!s->dPeerParts) HIPCHK(hipMalloc((void**)&s->dPeerParts, W * sizeof(double*)));
    HIPCHK(hipMemcpy((void*)s->dPeerParts, h.data(), W * sizeof(double*), hipMemcpyHostToDevice));
    HIPCHK(launch_sum_rank_chunks(s->dPeerParts, W, s->p.rank, s->S, s->dF, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    s->rs_pending = false;
    return 0;
}

// fold pending force partials into F (consumers other than the substep kernels)
static int settle_forces(mdqt_ctx* s) {
    if (local_reduce(s)) return -1;
    if (!s->f_pending) return 0;
    HIPCHK(launch_reduce_segments(s->dFpart, s->dF, s->pend_nseg, s->nloc, s->S, 3, s->stream));
    s->f_pending = false;
    return 0;
}

// Timing events only measure: no system-scope release/acquire when they complete.  With the
// default flags every timed launch ended in an L2 write-back + invalidate that cost the MD step
// ~20 us (kernel trace of the driver's bench command: gaps of 6.5 / 8.9 / 4.8 us around each
// timed pair of launches, none elsewhere).
static constexpr unsigned kTimingEventFlags = hipEventDisableSystemFence;

// record the next timing event of kind k (start/stop alternate)
static int mark(mdqt_ctx* s, int k) {
    auto& pool = s->evpool[k];
    if (s->evused[k] == (int)pool.size()) {
        hipEvent_t e;
        HIPCHK(hipEventCreateWithFlags(&e, kTimingEventFlags));
        pool.push_back(e);
    }
    HIPCHK(hipEventRecord(pool[s->evused[k]++], s->stream));
    return 0;
}

// a start/stop pair from the pool of kind k, for a launch that records them itself
static int take_events(mdqt_ctx* s, int k, hipEvent_t* e0, hipEvent_t* e1) {
    auto& pool = s->evpool[k];
    while ((int)pool.size() < s->evused[k] + 2) {
        hipEvent_t e;
        HIPCHK(hipEventCreateWithFlags(&e, kTimingEventFlags));
        pool.push_back(e);
    }
    *e0 = pool[s->evused[k]++];
    *e1 = pool[s->evused[k]++];
    return 0;
}

// force-call breakdown (timing kind bit 3): one event recorded now on the context stream, from the free list
static hipEvent_t bd_event(mdqt_ctx* s) {
    hipEvent_t e = nullptr;
    if (!s->bdfree.empty()) { e = s->bdfree.back(); s->bdfree.pop_back(); }
    else if (hipEventCreateWithFlags(&e, kTimingEventFlags) != hipSuccess) return nullptr;
    if (hipEventRecord(e, s->stream) != hipSuccess) { s->bdfree.push_back(e); return nullptr; }
    return e;
}
// will the next force call be timed (its tcount not yet advanced)?
static bool force_timed_next(const mdqt_ctx* s) {
    return s->timing && (s->tkinds & 1u) && (s->tkinds & 8u) && (s->tcount[0] % s->tperiod == s->toffset);
}

// the block kernel's work by tile-pair class for the current positions (k_n3b_census): out[0, 12)
// lane-steps, out[12, 24) distinct ion pairs — this rank's block pairs (diagnostic, outside any
// timed region: it runs the spatial order itself)
extern "C" int mdqt_force_census(mdqt_ctx* s, double* out, int n) {
    if (!s || !out) return fail("mdqt_force_census: NULL argument");
    if (n < 2 * kCensus) return fail("mdqt_force_census: need %d doubles", 2 * kCensus);
    if (!s->use_n3b || !s->sort_mode) return fail("mdqt_force_census: Newton-3 blocks in spatial order only");
    HIPCHK(hipSetDevice(s->dev));
    N3BArgs a;
    if (n3b_args(s, a)) return -1;
    unsigned long long* d = nullptr;
    unsigned long long h[2 * kCensus];
    HIPCHK(hipMalloc(&d, sizeof h));
    hipError_t e = launch_n3b_census(a, d, s->stream);
    if (e == hipSuccess) e = hipMemcpyAsync(h, d, sizeof h, hipMemcpyDeviceToHost, s->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    (void)hipFree(d);
    if (e != hipSuccess) return fail("mdqt_force_census: %s", hipGetErrorString(e));
    for (int k = 0; k < 2 * kCensus; ++k) out[k] = (double)h[k];
    return 0;
}

// the lock-step J loop's balance over a workgroup's 8 waves for the current positions (k_n3b_census, bal):
// out[0] the estimated VALU instructions of all tile pairs, out[1] the sum over J steps of 8 x the busiest
// wave's, out[2] the J steps with work — out[1] / out[0] is the excess of max over mean (diagnostic)
extern "C" int mdqt_force_jstep_balance(mdqt_ctx* s, double* out, int n) {
    if (!s || !out) return fail("mdqt_force_jstep_balance: NULL argument");
    if (n < 3) return fail("mdqt_force_jstep_balance: need 3 doubles");
    // (out[3..5] when n >= 6: 8 x the J-step pairs' best two-sub-step schedule, 8 x the same pairs in
    // lock-step, 8 x the per-(P, db) busiest wave's 8-step sum — see k_n3b_census)
    if (!s->use_n3b || !s->sort_mode) return fail("mdqt_force_jstep_balance: Newton-3 blocks in spatial order only");
    HIPCHK(hipSetDevice(s->dev));
    N3BArgs a;
    if (n3b_args(s, a)) return -1;
    unsigned long long* d = nullptr;
    unsigned long long h[11];
    HIPCHK(hipMalloc(&d, (2 * kCensus + 11) * sizeof(unsigned long long)));
    hipError_t e = launch_n3b_census(a, d, s->stream, nullptr, d + 2 * kCensus);
    if (e == hipSuccess) e = hipMemcpyAsync(h, d + 2 * kCensus, sizeof h, hipMemcpyDeviceToHost, s->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    (void)hipFree(d);
    if (e != hipSuccess) return fail("mdqt_force_jstep_balance: %s", hipGetErrorString(e));
    out[0] = (double)h[0]; out[1] = 8. * (double)h[1]; out[2] = (double)h[2];
    if (n >= 6) { out[3] = 8. * (double)h[3]; out[4] = 8. * (double)h[4]; out[5] = 8. * (double)h[5]; }
    // (out[6..8] when n >= 9: 4 waves on two I tiles each — heavy-light pairing, (q, 7 - q), (q, q + 4) —
    // 4 x the sum over J steps of the busiest wave's pair)
    if (n >= 9) { out[6] = 4. * (double)h[6]; out[7] = 4. * (double)h[7]; out[8] = 4. * (double)h[8]; }
    if (n >= 10) out[9] = 4. * (double)h[9];       // each J step paired heavy-light on its own
    if (n >= 11) out[10] = 4. * (double)h[10];     // the best of the 105 pairings per (P, db)
    return 0;
}

// the block kernel's evaluated lane-steps per block of this rank for the current positions (k_n3b_census's
// per-block sums): out[P - Plo], P = Plo .. Phi - 1 (*nblocks = Phi - Plo) — what each block's workgroups
// do; at world 1 every block, so the work of any rank partition follows
extern "C" int mdqt_force_block_work(mdqt_ctx* s, double* out, int n, int* nblocks) {
    if (!s || !out || !nblocks) return fail("mdqt_force_block_work: NULL argument");
    if (!s->use_n3b || !s->sort_mode) return fail("mdqt_force_block_work: Newton-3 blocks in spatial order only");
    const int nb = std::max(s->n3b.Phi - s->n3b.Plo, 0);
    *nblocks = nb;
    if (n < nb) return fail("mdqt_force_block_work: need %d doubles", nb);
    if (nb == 0) return 0;
    HIPCHK(hipSetDevice(s->dev));
    N3BArgs a;
    if (n3b_args(s, a)) return -1;
    unsigned long long* d = nullptr;
    HIPCHK(hipMalloc(&d, (2 * kCensus + (size_t)nb) * sizeof(unsigned long long)));
    std::vector<unsigned long long> h((size_t)nb);
    hipError_t e = launch_n3b_census(a, d, s->stream, d + 2 * kCensus);
    if (e == hipSuccess) e = hipMemcpyAsync(h.data(), d + 2 * kCensus, (size_t)nb * sizeof(unsigned long long),
                                            hipMemcpyDeviceToHost, s->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    (void)hipFree(d);
    if (e != hipSuccess) return fail("mdqt_force_block_work: %s", hipGetErrorString(e));
    for (int k = 0; k < nb; ++k) out[k] = (double)h[k];
    return 0;
}

// Sharded Newton-3 blocks: the ranks' block ranges by work.  The blocks' evaluated
// lane-steps vary several-fold along the Hilbert order (N = 1M: 0.49 .. 1.52 of the mean), and equal
// block counts left world 8 at 1.13 x the mean work on its busiest rank (world 2 and 4: 1.002;
// profiles/r05a_load_balance.json).  Once per size, at the first sharded force call (positions
// gathered): the census of EVERY block (k_n3b_census; integer counts, so every rank computes the same
// numbers from the same positions), then rank r takes the blocks [c_r, c_r+1) whose prefix work is
// nearest r / W of the total.  Any partition covers every block pair exactly once (the ownership is by
// P alone; tests/test_n3b_protocol.py); only the partial sums' order changes with it.
static int n3b_balance(mdqt_ctx* s) {
    const int W = s->p.world_size;
    if (s->balanced || W == 1 || !s->use_n3b || !s->sort_mode) return 0;
    s->balanced = true;
    N3BArgs& b = s->n3b;
    const int NB = b.NB;
    if (NB < W) return 0;
    N3BArgs a;
    if (n3b_args(s, a)) return -1;                  // (the spatial order and boxes of these positions)
    a.Plo = 0; a.Phi = NB;
    unsigned long long* d = nullptr;
    HIPCHK(hipMalloc(&d, (2 * kCensus + (size_t)NB) * sizeof(unsigned long long)));
    std::vector<unsigned long long> w((size_t)NB);
    hipError_t e = launch_n3b_census(a, d, s->stream, d + 2 * kCensus);
    if (e == hipSuccess) e = hipMemcpyAsync(w.data(), d + 2 * kCensus, (size_t)NB * sizeof(unsigned long long),
                                            hipMemcpyDeviceToHost, s->stream);
    if (e == hipSuccess) e = hipStreamSynchronize(s->stream);
    (void)hipFree(d);
    if (e != hipSuccess) return fail("force balance census: %s", hipGetErrorString(e));
    std::vector<double> pre((size_t)NB + 1, 0.);
    for (int k = 0; k < NB; ++k) pre[k + 1] = pre[k] + (double)w[k];
    const double tot = pre[NB];
    std::vector<int> cut((size_t)W + 1, 0);
    cut[W] = NB;
    for (int r = 1; r < W; ++r) {
        const double t = tot * r / W;
        int k = (int)(std::lower_bound(pre.begin(), pre.end(), t) - pre.begin());   // pre[k] >= t
        if (k > 0 && t - pre[k - 1] < pre[k] - t) --k;                             // the nearer boundary
        cut[r] = std::min(std::max(k, cut[r - 1] + 1), NB - (W - r));               // >= 1 block per rank
    }
    auto ratio = [&](const std::vector<int>& c) {
        double mx = 0.;
        for (int r = 0; r < W; ++r) mx = std::max(mx, pre[c[r + 1]] - pre[c[r]]);
        return tot > 0. ? mx / (tot / W) : 1.;
    };
    std::vector<int> eq((size_t)W + 1);
    for (int r = 0; r <= W; ++r) eq[r] = (int)((long)r * NB / W);
    s->balance_ratio_eq = ratio(eq);
    if (s->balance_opt) {
        s->balance_ratio = ratio(cut);
        n3b_set_range(b, cut[s->p.rank], cut[s->p.rank + 1]);
        if (ensure_aux(s)) return -1;               // (the runs, hence the i-slots, follow the range)
    } else {
        s->balance_ratio = s->balance_ratio_eq;
    }
    return 0;
}

extern "C" int mdqt_forces(mdqt_ctx* s) {                 // forces(), SpeedUp:192-236
    if (!s) return fail("NULL context");
    if (s->nloc == 0) return 0;
    HIPCHK(hipSetDevice(s->dev));
    const bool tm = s->timing && (s->tkinds & 1u) && (s->tcount[0]++ % s->tperiod == s->toffset);
    // timing: the Newton-3 tile kernel (one launch) records its own timestamps; the other
    // schemes (several kernels, collectives) are bracketed by events on the stream
    const bool tm_marks = tm && !s->use_n3;
    if (tm_marks && mark(s, 0)) return -1;
    if (s->use_n3) {
        N3Args a{};                  // variant 2 (MCMD's exact pair set, rc2) is not used here
        if (s->force_variant > 1) return fail("mdqt_forces: force_kernel must be 0 or 1");
        // one tile (N <= 64): its one slot has F's [3][S] layout, so the kernel writes F itself and
        // nothing is pending (the substep kernels read F when nseg == 1)
        const bool one_slot = s->nslots == 1;
        // the split table (ensure_aux) unless the MD steps count tile arrivals (options overlap, fused_step:
        // then every force call of the context takes the plain table)
        const bool split = s->nsplit > 0 && !s->force_arrive && !one_slot && !s->overlap_opt && !s->fused_opt;
        a.R = s->dR; a.P = one_slot ? s->dF : s->dFpart; a.pairs = split ? s->dPairs + s->npairs : s->dPairs;
        a.N = s->N; a.S = s->S; a.ntiles = (s->N + 63) / 64; a.npairs = split ? s->nsplit_wg : s->npairs;
        ForceArgs c = force_args(s, nullptr);
        a.L = c.L; a.lDeb = c.lDeb; a.Rcut = c.Rcut; a.invlDeb = c.invlDeb; a.micT = c.micT;
        a.micGuard = c.micGuard;
        a.guard = c.guard;
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (tm && take_events(s, 0, &e0, &e1)) return -1;
        a.arrive = s->force_arrive;                // overlapped MD step: count finished workgroups
        HIPCHK(launch_forces_n3(a, s->force_variant, s->stream, e0, e1));
        s->f_pending = !one_slot;  // slots summed by the next substep launch (or settle_forces)
        s->pend_nseg = s->nslots + (split ? split_slots(s) : 0);
    } else if (s->use_n3b) {
        const bool bd = tm && (s->tkinds & 8u);    // the breakdown of this call
        mdqt_ctx::BdCall bc;
        if (bd) {
            bc.ag0 = s->bd_ag[0]; bc.ag1 = s->bd_ag[1];
            bc.m[0] = bd_event(s);
        }
        s->bd_ag[0] = s->bd_ag[1] = nullptr;
        if (n3b_balance(s)) return -1;
        N3BArgs a;
        if (n3b_args(s, a)) return -1;
        if (bd) bc.m[1] = bd_event(s);
        const int W = s->p.world_size;
        if (a.tailb) {
            HIPCHK(hipMemsetAsync(a.tailb, 0, (size_t)4 * a.T * sizeof(double), s->stream));
            HIPCHK(hipMemsetAsync(s->dTailSt + 3, 0, sizeof(unsigned long long), s->stream));
        }
        hipEvent_t e0 = nullptr, e1 = nullptr;     // timed call: the block kernel alone as well
        if (tm && take_events(s, 2, &e0, &e1)) return -1;
        hipEvent_t pm[3] = {nullptr, nullptr, nullptr};   // after the plan, the kernel, the reduction
        if (bd)
            for (auto& e : pm) {
                if (!s->bdfree.empty()) { e = s->bdfree.back(); s->bdfree.pop_back(); }
                else HIPCHK(hipEventCreateWithFlags(&e, kTimingEventFlags));
            }
        HIPCHK(launch_forces_n3b(a, s->force_variant, W == 1 ? s->dF : s->dFr, s->stream, e0, e1, bd ? pm : nullptr));
        if (bd) { bc.m[2] = pm[0]; bc.m[3] = pm[1]; bc.m[4] = pm[2]; }
        if (a.tailb) {                  // measured tail: complete the per-tile sums, then enforce eps
            if (W > 1 && s->comm) {
                NCCLCHK(ncclAllReduce(a.tailb, a.tailb, (size_t)4 * a.T, ncclDouble, ncclSum, s->comm, s->stream));
            }
            if (W == 1 || s->comm) {
                if (tail_enforce(s, a, W == 1 ? s->dF : s->dFr)) return -1;
            } else {                    // in-process group: once every rank has its sums (local_reduce)
                s->tail_pending = true;
                s->tail_args = a;
            }
        }
        if (bd) bc.m[5] = bd_event(s);
        if (W > 1) {
            if (s->comm) {
                NCCLCHK(ncclReduceScatter(s->dFr, s->dF, (size_t)3 * s->S, ncclDouble, ncclSum, s->comm, s->stream));
            } else if (!s->local.empty()) {
                s->rs_pending = true;      // formed by local_reduce once every rank has its partials
            } else {
                return fail("mdqt_forces: sharded Newton-3 blocks need a communicator (mdqt_comm_init)");
            }
        }
        if (bd) {
            bc.m[6] = bd_event(s);
            s->bdcalls.push_back(bc);
        }
        s->f_pending = false;
    } else if (s->nseg == 1) {
        HIPCHK(launch_forces(force_args(s, s->dF), s->stream));
    } else {
        HIPCHK(launch_forces(force_args(s, s->dFpart), s->stream));
        s->f_pending = true;       // summed by the next substep launch (or settle_forces)
        s->pend_nseg = s->nseg;
    }
    if (tm_marks && mark(s, 0)) return -1;
    return 0;
}

// n substeps of (step if do_step; qstep if do_qt_flag) — t advances only when advance_t
static int run_substeps(mdqt_ctx* s, int n, int do_step, int do_qt_flag, int advance_t) {
    if (local_reduce(s)) return -1;
    HIPCHK(hipSetDevice(s->dev));
    const int do_qt = do_qt_flag && s->p.qt_enabled;
    if (do_qt && s->p.qt_model != 0 && s->qt_math != 2) return fail("the optical-pumping qt_models need qt_math 2");
    const bool d48 = do_qt && s->p.rng_mode == 0;
    while (n > 0) {
        const int m = d48 ? 1 : (n < MAXSUB ? n : MAXSUB);   // drand48: the stream orders ions per substep
        SubstepArgs a;
        memset(&a, 0, sizeof a);
        a.R = s->dR + (size_t)s->p.rank * 3 * s->S;
        a.V = s->dV; a.F = s->dF; a.psi = s->dPsi; a.tPart = s->dTp;
        a.Fpart = s->dFpart; a.nseg = s->f_pending ? s->pend_nseg : 1;
        a.oor = s->dFlags;
        if (s->sub_stream) {                            // overlapped MD step (mdqt_md_steps)
            a.arrive = s->dArrive;
            a.arrive_target = s->sub_target;
            a.spin_err = s->dSpinErr;
            a.arrive_sleep = 2;
        }
        s->f_pending = false;
        a.n = s->nloc; a.S = s->S; a.gid0 = (uint64_t)s->lo;
        a.q0 = s->qidx;
        a.nsub = m; a.do_step = do_step; a.do_qt = do_qt;
        a.L = s->L;
        a.qc = s->qc;
        double t = s->t;
        a.movmask = 0;
        a.expdet_zero = 1;
        for (int k = 0; k < m; ++k) {
            a.t[k] = t;
            a.expDet[k] = expDetuning_of(&s->p, t);
            if (t > 0) a.movmask |= 1u << k;
            if (a.expDet[k] != 0.) a.expdet_zero = 0;
            if (advance_t) t += s->dtQ;                    // qstep: t += dtQuant (:716)
        }
        if (d48 && s->nloc > 0) {
            D48Args r;
            r.psi = s->dPsi; r.n = s->nloc; r.S = s->S;
            r.state = s->dX48; r.jA = s->dX48 + 1; r.jC = s->dX48 + 49;
            r.U = s->dU; r.qc = s->qc; r.fast = s->qt_math;
            HIPCHK(launch_d48_resolve(r, s->stream));
            a.U = s->dU;
        }
        const bool tm = s->timing && (s->tkinds & 2u) && (s->tcount[1]++ % s->tperiod == s->toffset);
        hipEvent_t e0 = nullptr, e1 = nullptr;       // timing: the kernel's own timestamps
        if (tm && (take_events(s, 1, &e0, &e1))) return -1;
        hipStream_t st = s->sub_stream ? s->sub_stream : s->stream;
        int inst = 0;
        if (s->qt_math == 2) HIPCHK(launch_substeps_r(a, s->dFTab, s->sub_stream ? 2 : s->substep_mode, st, e0, e1, &inst));
        else HIPCHK(launch_substeps(a, s->dTab, s->substep_mode, s->qt_math, s->stream, e0, e1, &inst));
        s->last_qt_kernel = inst;
        s->last_qt_nseg = a.nseg;
        if (advance_t) {
            s->t = t;
            s->qidx += (uint64_t)m;
        }
        n -= m;
    }
    return 0;
}

// measureSpinUps / tagParticles of the optical-pumping programs (see include/mdqt.h)
extern "C" int mdqt_tag_spin_up(mdqt_ctx* s, int* tags, int* n_up) {
    if (!s) return fail("NULL context");
    if (s->p.qt_model == 0) return fail("mdqt_tag_spin_up: qt_model 0 (laser cooling) has no spin tagging");
    HIPCHK(hipSetDevice(s->dev));
    const int n = s->nloc;
    int* d = nullptr;
    if (n > 0) {
        HIPCHK(hipMalloc(&d, (size_t)n * sizeof(int)));
        HIPCHK(launch_tag_spin_up(s->dPsi, n, s->S, (uint64_t)s->lo, s->qidx, s->qc, d, s->stream));
    }
    std::vector<int> h((size_t)n, 0);
    if (n > 0) {
        HIPCHK(hipMemcpyAsync(h.data(), d, (size_t)n * sizeof(int), hipMemcpyDeviceToHost, s->stream));
        HIPCHK(hipStreamSynchronize(s->stream));
        HIPCHK(hipFree(d));
    }
    int cnt = 0;
    for (int i = 0; i < n; ++i) cnt += h[i];
    if (tags)
        for (int i = 0; i < n; ++i) tags[s->lo + i] = h[i];
    if (n_up) *n_up = cnt;
    return 0;
}

extern "C" int mdqt_step(mdqt_ctx* s) { return s ? run_substeps(s, 1, 1, 0, 0) : fail("NULL context"); }
extern "C" int mdqt_qstep(mdqt_ctx* s) { return s ? run_substeps(s, 1, 0, 1, 1) : fail("NULL context"); }
extern "C" int mdqt_substeps(mdqt_ctx* s, int n) {
    if (!s) return fail("NULL context");
    if (n < 0) return fail("negative substep count");
    return run_substeps(s, n, 1, 1, 1);
}

// The overlapped MD step applies to one unsharded system on the Newton-3 tile scheme with the
// lane-per-state QT kernel (qt_math 2, Philox stream), one fused launch per MD interval.
static bool overlap_applies(const mdqt_ctx* s) {
    return s->overlap_opt && s->p.world_size == 1 && s->local.empty() && s->use_n3 && s->nslots > 1 && s->qt_math == 2 &&
           s->p.qt_enabled && s->p.rng_mode == 1 && s->ratio <= MAXSUB && s->nloc > 0 &&
           (s->substep_mode == 2 || (s->substep_mode == 0 && s->nloc < kLaneKernelMaxIons));
}

// per-tile arrival counters of the overlapped / fused MD step (monotonic: a launch adds T to
// every tile's counter, the waiters compare with the running epoch)
static int arrive_setup(mdqt_ctx* s) {
    const int T = (s->N + 63) / 64;
    if (s->dArrive && s->arriveCap >= T) return 0;
    HIPCHK(hipStreamSynchronize(s->stream));
    if (s->qs) HIPCHK(hipStreamSynchronize(s->qs));
    if (s->dArrive) HIPCHK(hipFree(s->dArrive));
    s->dArrive = nullptr;
    HIPCHK(hipMalloc(&s->dArrive, (size_t)T * sizeof(unsigned long long)));
    HIPCHK(hipMemset(s->dArrive, 0, (size_t)T * sizeof(unsigned long long)));
    if (!s->dSpinErr) {
        HIPCHK(hipMalloc(&s->dSpinErr, sizeof(int)));
        HIPCHK(hipMemset(s->dSpinErr, 0, sizeof(int)));
    }
    HIPCHK(hipDeviceSynchronize());
    s->arriveCap = T;
    s->arriveEpoch = 0;
    return 0;
}

static int overlap_setup(mdqt_ctx* s) {
    if (arrive_setup(s)) return -1;
    if (s->qs) return 0;
    HIPCHK(hipStreamCreateWithFlags(&s->qs, hipStreamNonBlocking));
    HIPCHK(hipEventCreateWithFlags(&s->evQ, hipEventDisableTiming | hipEventDisableSystemFence));
    HIPCHK(hipEventCreateWithFlags(&s->evS, hipEventDisableTiming | hipEventDisableSystemFence));
    return 0;
}

// MD steps with the force and QT launches overlapped: step k's force launch (context stream)
// waits for step k-1's QT launch by an event; step k's QT launch (its own stream, in order after
// step k-1's) starts at once, issues its prologue loads and Philox draws while the forces are
// computed, and waits on the device until the tile pairs of its ions' tile have arrived.  Same
// kernels, same operations: bit-identical to the sequential order (tests/test_gpu_parity.py).
// Measured at C2 (one MI355X): 104-107 us per MD step against 45.6 sequential — the two
// cross-stream event waits cost ~17 us per step by themselves, and the resident QT waves (176
// VGPRs) leave room for 1,344 of the force launch's 1,596 workgroups, so it runs in two rounds
// (17.6 -> 52-70 us).  Kept as an option (default off) with its bit-identity test.
static int md_steps_overlapped(mdqt_ctx* s, int n) {
    if (overlap_setup(s)) return -1;
    HIPCHK(hipEventRecord(s->evS, s->stream));
    HIPCHK(hipStreamWaitEvent(s->qs, s->evS, 0));
    for (int k = 0; k < n; ++k) {
        if (k > 0) HIPCHK(hipStreamWaitEvent(s->stream, s->evQ, 0));
        if (k > 0 && k % 64 == 0 && check_range_flag(s)) return -1;
        s->force_arrive = s->dArrive;
        const int rc = mdqt_forces(s);
        s->force_arrive = nullptr;
        if (rc) return -1;
        s->arriveEpoch += (unsigned long long)((s->N + 63) / 64);   // T tile pairs touch every tile
        s->c0++;
        s->sub_stream = s->qs;
        s->sub_target = s->arriveEpoch;
        const int rq = run_substeps(s, s->ratio, 1, 1, 1);
        s->sub_stream = nullptr;
        if (rq) return -1;
        HIPCHK(hipEventRecord(s->evQ, s->qs));
    }
    HIPCHK(hipStreamWaitEvent(s->stream, s->evQ, 0));      // later work on the context stream
    return 0;
}

// One MD step as ONE launch (mdqt_qtfast.hip k_md_step): the Newton-3 tile pairs of forces() and
// the interval's fused substeps, the QT workgroups waiting on the device for the arrival counts
// of their ions' tiles instead of a kernel boundary.  Applies to one unsharded system on the tile
// scheme with the lane QT kernel's FAST instance (qt_math 2, Philox, t > 0, the whole interval in
// one launch, no range guard).  Same operations as forces() + substeps(ratio): bit-identical.
// Measured at C2 (one MI355X, per-workgroup stamps `tools/md_stamps.py`): 56-63 us per MD step
// against 43.5 for the two launches — one kernel has one VGPR count, so the tile pairs run with
// the QT part's 162 (3 waves per SIMD instead of 7), the QT workgroups dispatched while the last
// tile pairs still run take their CU slots, and the substep loops of early-complete tiles compete
// with the remaining tile pairs; the force work ends at 32-37 us instead of 18.  Kept as an option
// (default off) with its bit-identity tests.
static bool fused_applies(mdqt_ctx* s) {
    if (!(s->fused_opt && !s->overlap_opt && s->p.world_size == 1 && s->local.empty() && s->use_n3 && s->nslots > 1 &&
          s->qt_math == 2 && s->p.qt_enabled && s->p.rng_mode == 1 && s->ratio <= MAXSUB && s->nloc > 0 &&
          s->t > 0 && s->force_variant <= 1 &&
          (s->substep_mode == 2 || (s->substep_mode == 0 && s->nloc < kLaneKernelMaxIons))))
        return false;
    return !force_args(s, nullptr).guard;
}

static int md_step_fused(mdqt_ctx* s) {
    if (arrive_setup(s)) return -1;
    HIPCHK(hipSetDevice(s->dev));
    const unsigned long long T = (unsigned long long)((s->N + 63) / 64);
    N3Args f{};
    const ForceArgs c = force_args(s, nullptr);
    f.R = s->dR; f.P = s->dFpart; f.pairs = s->dPairs;
    f.N = s->N; f.S = s->S; f.ntiles = (int)T; f.npairs = s->npairs;
    f.L = c.L; f.lDeb = c.lDeb; f.Rcut = c.Rcut; f.invlDeb = c.invlDeb; f.micT = c.micT;
    f.micGuard = c.micGuard; f.guard = 0;
    f.arrive = s->dArrive;
    SubstepArgs a;                                     // as run_substeps(s, ratio, 1, 1, 1)
    memset(&a, 0, sizeof a);
    const int m = s->ratio;
    a.R = s->dR; a.V = s->dV; a.F = s->dF; a.psi = s->dPsi; a.tPart = s->dTp;
    a.Fpart = s->dFpart; a.nseg = s->nslots;
    a.oor = s->dFlags;
    a.arrive = s->dArrive;
    a.arrive_target = s->arriveEpoch + T;
    a.spin_err = s->dSpinErr;
    a.arrive_sleep = 2;
    a.n = s->nloc; a.S = s->S; a.gid0 = (uint64_t)s->lo;
    a.q0 = s->qidx;
    a.nsub = m; a.do_step = 1; a.do_qt = 1;
    a.L = s->L;
    a.qc = s->qc;
    double t = s->t;
    a.movmask = 0;
    a.expdet_zero = 1;
    for (int k = 0; k < m; ++k) {
        a.t[k] = t;
        a.expDet[k] = expDetuning_of(&s->p, t);
        if (t > 0) a.movmask |= 1u << k;
        if (a.expDet[k] != 0.) a.expdet_zero = 0;
        t += s->dtQ;                                   // qstep: t += dtQuant (:716)
    }
    if (a.movmask != (m >= 32 ? 0xFFFFFFFFu : (1u << m) - 1u)) return fail("md_step_fused: t <= 0 in the interval");
    const bool tm = s->timing && (s->tkinds & 2u) && (s->tcount[1]++ % s->tperiod == s->toffset);
    hipEvent_t e0 = nullptr, e1 = nullptr;
    if (tm && take_events(s, 1, &e0, &e1)) return -1;
    HIPCHK(launch_md_step(f, a, s->dFTab, s->force_variant, s->stream, e0, e1));
    s->last_qt_kernel = QTK_MD_STEP;
    s->last_qt_nseg = a.nseg;
    s->arriveEpoch += T;
    s->f_pending = false;                              // F written by the QT workgroups
    s->t = t;
    s->qidx += (uint64_t)m;
    return 0;
}

extern "C" int mdqt_md_steps(mdqt_ctx* s, int n) {
    if (!s) return fail("NULL context");
    if (n > 0 && overlap_applies(s)) return md_steps_overlapped(s, n);
    for (int k = 0; k < n; ++k) {
        if (k > 0 && k % 64 == 0 && check_range_flag(s)) return -1;
        if (fused_applies(s)) {
            if (local_reduce(s) || md_step_fused(s)) return -1;
            s->last_fused = 1;
            s->c0++;
            continue;
        }
        s->last_fused = 0;
        if (mdqt_allgather_positions(s)) return -1;     // sharded: other slabs' R
        if (mdqt_forces(s)) return -1;
        s->c0++;
        if (mdqt_substeps(s, s->ratio)) return -1;
    }
    return 0;
}

// stateless pair kernels on host arrays (tests, and the MD-only programs' force seam)
static int pairs_raw(int mode, int N, double L, double lDeb, const double* R, size_t ld, double* out,
                     int nseg_req, int device, int variant) {
    if (N < 1 || !R || !out || ld < (size_t)N) return fail("pairs_raw: bad arguments");
    if (variant < 0 || variant > 1) return fail("pairs_raw: variant must be 0 (exact) or 1 (fast)");
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev < 1) return fail("no HIP device available");
    if (device >= 0) HIPCHK(hipSetDevice(device));
    int lo, hi, S;
    if (mdqt_slab(N, 1, 0, &lo, &hi, &S)) return -1;
    mdqt_ctx tmp;                                   // only for choose_segments
    memset(&tmp.p, 0, sizeof tmp.p);
    tmp.p.world_size = 1;
    tmp.scheme_opt = 1;
    tmp.N = N; tmp.p.force_segments = nseg_req;
    choose_segments(&tmp);
    const int nseg = tmp.nseg;
    std::vector<double> h((size_t)3 * S, 0.);
    for (int c = 0; c < 3; ++c)
        for (int i = 0; i < N; ++i) h[(size_t)c * S + i] = R[(size_t)c * ld + i];
    double *dR = nullptr, *dP = nullptr, *dO = nullptr;
    hipStream_t st;
    HIPCHK(hipStreamCreate(&st));
    HIPCHK(hipMalloc(&dR, h.size() * sizeof(double)));
    HIPCHK(hipMalloc(&dP, (size_t)3 * S * nseg * sizeof(double)));
    HIPCHK(hipMalloc(&dO, (size_t)3 * S * sizeof(double)));
    HIPCHK(hipMemcpyAsync(dR, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice, st));
    int oor = 0;
    for (size_t k = 0; k < (size_t)3 * N && !oor; ++k) {
        const double x = R[(k / N) * ld + k % N];
        if (!(x >= -0.125 * L && x <= 1.125 * L)) oor = 1;
    }
    ForceArgs a;
    a.Rall = dR; a.Fpart = dP; a.N = N; a.S = S; a.row_lo = 0; a.nrows = N;
    a.nseg = nseg; a.seglen = tmp.seglen;
    fill_pair_consts(a, L, lDeb, variant);
    a.guard = oor;
    HIPCHK(mode == 0 ? launch_forces(a, st) : launch_potential_rows(a, st));
    HIPCHK(launch_reduce_segments(dP, dO, nseg, N, S, mode == 0 ? 3 : 1, st));
    HIPCHK(hipMemcpyAsync(h.data(), dO, h.size() * sizeof(double), hipMemcpyDeviceToHost, st));
    HIPCHK(hipStreamSynchronize(st));
    HIPCHK(hipFree(dR)); HIPCHK(hipFree(dP)); HIPCHK(hipFree(dO));
    HIPCHK(hipStreamDestroy(st));
    if (mode == 0) {
        for (int c = 0; c < 3; ++c)
            for (int i = 0; i < N; ++i) out[(size_t)c * ld + i] = h[(size_t)c * S + i];
    } else {
        for (int i = 0; i < N; ++i) out[i] = h[i];
    }
    return 0;
}

extern "C" int mdqt_forces_raw(int N, double L, double lDeb, const double* R, size_t ld, double* F,
                               int nseg, int device, int variant) {
    return pairs_raw(0, N, L, lDeb, R, ld, F, nseg, device, variant);
}

extern "C" int mdqt_potentials_raw(int N, double L, double lDeb, const double* R, size_t ld, double* U,
                                   int nseg, int device, int variant) {
    return pairs_raw(1, N, L, lDeb, R, ld, U, nseg, device, variant);
}

// ---------------------------------------------------------------------------------------------
// observables (Epotential :244-281, output :917-1032)
// ---------------------------------------------------------------------------------------------

// device: scratch[0] = sum over owned rows of the full-row pair potential.  World 1, partials up
// to 64 MB: the potential rows get a buffer of their own, so pending force slots stay pending
// (the next substep launch sums them in its prologue: no reduce launch, and that launch stays the
// production instance); otherwise they reuse the force partials after settling them.
static int potential_rows(mdqt_ctx* s, double* urow_dev) {
    if (s->nloc == 0) return 0;
    // world 1 with the Newton-3 tile scheme: each distinct pair's potential once (the tile kernel's
    // POT mode), the ntiles slots of component 0 summed per ion (half the pair evaluations of the
    // rows; the same per-ion row sums up to summation order)
    if (s->use_n3 && !s->use_n3b && s->p.world_size == 1 && s->local.empty() && s->force_variant <= 1 &&
        s->n3_potential) {
        const size_t need = (size_t)s->nslots * s->S;   // one plane per slot (component 0)
        if (need > s->capUpart) {
            if (s->dUpart) HIPCHK(hipFree(s->dUpart));
            s->dUpart = nullptr;
            s->capUpart = 0;
            HIPCHK(hipMalloc(&s->dUpart, need * sizeof(double)));
            s->capUpart = need;
        }
        N3Args a{};
        a.R = s->dR; a.P = s->dUpart; a.pairs = s->dPairs;
        a.N = s->N; a.S = s->S; a.ntiles = (s->N + 63) / 64; a.npairs = s->npairs;
        ForceArgs c = force_args(s, nullptr);
        a.L = c.L; a.lDeb = c.lDeb; a.Rcut = c.Rcut; a.invlDeb = c.invlDeb; a.micT = c.micT;
        a.micGuard = c.micGuard;
        a.guard = c.guard;
        a.arrive = nullptr;
        HIPCHK(launch_potential_n3(a, s->force_variant, s->stream));
        HIPCHK(launch_reduce_segments(s->dUpart, urow_dev, s->nslots, s->nloc, s->S, 1, s->stream, (size_t)s->S));
        return 0;
    }
    // world 1 with Newton-3 blocks (N > 65,536): the block kernel's POT mode, per-ion row sums by
    // k_n3b_reduce (the block slots are free between force calls: the force path reduces at once)
    // Round 6 (option potential_plan): on the force call's plan — the same skip radius,
    // sub-tile groups and error-bounded forms (pair_u_cut, the f32 ultra-far form), the same measured and
    // enforced tail (tiles whose sub-tile force sums exceed eps get their U_i recomputed exactly).  Since
    // u(r) < lDeb g(r) and each form's relative error on u is at most its error on the force, every U_i is
    // within lDeb x (the force call's per-ion bound: tail eps + the tiers') of its sum to L/2, and Epot =
    // sum U_i / 2N within half that (C4, N = 1M: ~1e-12 absolute on Epot ~ 5; north_star asks 1e-6
    // relative).  Tests: tests/test_gpu_large.py test_epotential_on_the_plan.
    if (s->use_n3b && s->p.world_size == 1 && s->local.empty() && s->force_variant <= 1 && s->n3_potential) {
        if (settle_forces(s)) return -1;
        N3BArgs a;
        if (n3b_args(s, a)) return -1;
        const bool planned = s->pot_plan && a.plan && s->force_variant == 1 && !a.guard;
        if (!planned) {
            a.plan = nullptr; a.tmask = nullptr; a.tmw = 0; a.tailb = nullptr;
            a.Rskip = a.Rcut;                       // (the no-plan kernel skips only beyond L/2 for potentials)
        } else if (a.tailb) {
            HIPCHK(hipMemsetAsync(a.tailb, 0, (size_t)4 * a.T * sizeof(double), s->stream));
            HIPCHK(hipMemsetAsync(s->dTailSt + 8 + 3, 0, sizeof(unsigned long long), s->stream));
        }
        hipEvent_t e0 = nullptr, e1 = nullptr;
        if (s->timing && (s->tkinds & 4u) && take_events(s, 3, &e0, &e1)) return -1;
        HIPCHK(launch_potential_n3b(a, s->force_variant, urow_dev, s->stream, e0, e1));
        if (a.tailb) {                              // the enforcement (its own counters: dTailSt[8, 16))
            HIPCHK(launch_tail_max(a.tailb, a.T, error_eps(s, a), s->dTailSt + 8, s->dTailList, s->stream));
            HIPCHK(launch_tail_fix(a, s->dTailSt + 8, s->dTailList, urow_dev, s->stream, true));
        }
        return 0;
    }
    double* buf = s->dFpart;
    const size_t need = (size_t)s->nseg * 3 * s->S;
    if (s->p.world_size == 1 && s->local.empty() && need * sizeof(double) <= ((size_t)64 << 20)) {
        if (need > s->capUpart) {
            if (s->dUpart) HIPCHK(hipFree(s->dUpart));
            s->dUpart = nullptr;
            s->capUpart = 0;
            HIPCHK(hipMalloc(&s->dUpart, need * sizeof(double)));
            s->capUpart = need;
        }
        buf = s->dUpart;
    } else if (settle_forces(s)) {
        return -1;
    }
    HIPCHK(launch_potential_rows(force_args(s, buf), s->stream));
    HIPCHK(launch_reduce_segments(buf, urow_dev, s->nseg, s->nloc, s->S, 1, s->stream));
    return 0;
}

extern "C" int mdqt_partial_observables(mdqt_ctx* s, double vxAvg, double out5[5], double* Pvel) {
    if (!s) return fail("NULL context");
    HIPCHK(hipSetDevice(s->dev));
    double* scr = s->dScr;           // [0] sum vx, [8] vxAvg, [16..19] sums, [64..] KDE bins
    if (potential_rows(s, s->dUrow)) return -1;
    HIPCHK(launch_sum_vx(s->dV, s->nloc, scr, s->stream));
    HIPCHK(hipMemcpyAsync(scr + 8, &vxAvg, sizeof(double), hipMemcpyHostToDevice, s->stream));
    HIPCHK(launch_energy_sums(s->dV, s->nloc, s->S, scr + 8, s->dUrow, scr + 16, s->stream));
    int nch = s->nloc / 32;                                 // cold ions sit in the first bins:
    if (nch < 1) nch = 1;                                    // short chunks spread that work
    if (nch > s->kdeChunks) nch = s->kdeChunks;
    double* Pout = scr + 64;
    if (s->nloc > 0) HIPCHK(launch_kde(s->dV, s->nloc, s->S, scr + 8, s->dKde, nch, Pout, s->stream));
    else HIPCHK(hipMemsetAsync(Pout, 0, 3 * NBINS * sizeof(double), s->stream));
    double h[64 + 3 * NBINS];
    HIPCHK(hipMemcpyAsync(h, scr, sizeof h, hipMemcpyDeviceToHost, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    out5[0] = s->nloc ? h[0] : 0.;
    out5[1] = s->nloc ? h[16] : 0.; out5[2] = s->nloc ? h[17] : 0.; out5[3] = s->nloc ? h[18] : 0.;
    out5[4] = s->nloc ? h[19] : 0.;
    if (Pvel) memcpy(Pvel, h + 64, 3 * NBINS * sizeof(double));
    return 0;
}

// the per-ion pair-potential row sums U_i that Epotential() adds up (world 1; by ion index): the same path as
// Epotential() (Newton-3 tiles or blocks — on the force call's plan unless potential_plan 0 — or rows)
extern "C" int mdqt_potential_rows(mdqt_ctx* s, double* U, int n) {
    if (!s || !U) return fail("mdqt_potential_rows: NULL argument");
    if (s->p.world_size != 1 || !s->local.empty()) return fail("mdqt_potential_rows: world 1 only");
    if (n < s->N) return fail("mdqt_potential_rows: need %d doubles", s->N);
    HIPCHK(hipSetDevice(s->dev));
    if (potential_rows(s, s->dUrow)) return -1;
    HIPCHK(hipMemcpyAsync(U, s->dUrow, (size_t)s->N * sizeof(double), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    return 0;
}

extern "C" int mdqt_epotential(mdqt_ctx* s, double* Epot) {   // Epotential(), :244-281
    if (!s) return fail("NULL context");
    double o[5];
    if (mdqt_allgather_positions(s)) return -1;          // collective when sharded
    if (mdqt_partial_observables(s, 0., o, nullptr)) return -1;
    if (mdqt_allreduce_sum(s, o, 5)) return -1;
    // sum_{i<j} u = (sum_i sum_{j != i} u) / 2 ; Epot /= N (:280)
    s->Epot = s->N > 0 ? (o[4] / 2.) / (double)s->N : 0.;
    if (Epot) *Epot = s->Epot;
    return 0;
}

// output()'s observables at world 1 in one device pass and one synchronisation: <vx> stays on
// the device (k_sum_vx writes sum / N for the energy sums and the KDE), the per-ion columns
// (vx, S / P / D populations) come from k_output_pack instead of a full wavefunction download.
// Same operations as the general path below (the populations: the host loop's order).
static int observables_w1(mdqt_ctx* s, double out7[7], double* Pvel, double* pops, double* vx) {
    const int N = s->N;
    double* scr = s->dScr;           // [0] sum vx, [8] vxAvg, [16..19] sums, [64..] KDE bins
    HIPCHK(hipSetDevice(s->dev));
    if (potential_rows(s, s->dUrow)) return -1;
    HIPCHK(launch_sum_vx(s->dV, N, scr, s->stream, scr + 8, N));
    HIPCHK(launch_energy_sums(s->dV, N, s->S, scr + 8, s->dUrow, scr + 16, s->stream));
    int nch = N / 32;
    if (nch < 1) nch = 1;
    if (nch > s->kdeChunks) nch = s->kdeChunks;
    HIPCHK(launch_kde(s->dV, N, s->S, scr + 8, s->dKde, nch, scr + 64, s->stream));
    const bool pack = pops || vx;
    if (pack) HIPCHK(launch_output_pack(s->dV, s->dPsi, N, s->S, s->p.qt_model, s->dPack, s->stream));
    std::vector<double> h(64 + 3 * NBINS), col(pack ? (size_t)4 * N : 0);
    HIPCHK(hipMemcpyAsync(h.data(), scr, h.size() * sizeof(double), hipMemcpyDeviceToHost, s->stream));
    if (pack) HIPCHK(hipMemcpyAsync(col.data(), s->dPack, col.size() * sizeof(double), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    const double velXAvg = h[8];
    const double EkinX = h[16] / (double)N, EkinY = h[17] / (double)N, EkinZ = h[18] / (double)N;   // :945-947
    s->Epot = (h[19] / 2.) / (double)N;                                                          // :948
    out7[0] = s->t; out7[1] = EkinX; out7[2] = EkinY; out7[3] = EkinZ; out7[4] = s->Epot;
    out7[5] = EkinX + EkinY + EkinZ + s->Epot - s->Epot0; out7[6] = velXAvg;                   // :954
    if (Pvel) {
        const double norm = (6.0 * sqrt(2 * M_PI * 0.002 * 0.002));                            // :975-978
        for (int j = 0; j < 3 * NBINS; ++j) Pvel[j] = h[64 + j] / norm;
    }
    if (vx) memcpy(vx, col.data(), (size_t)N * sizeof(double));
    if (pops)
        for (int i = 0; i < N; i++) {
            pops[3 * i + 0] = col[(size_t)N + i];
            pops[3 * i + 1] = col[2 * (size_t)N + i];
            pops[3 * i + 2] = col[3 * (size_t)N + i];
        }
    return 0;
}

static bool observables_w1_applies(const mdqt_ctx* s) {
    return s->p.world_size == 1 && s->local.empty() && s->N > 0 && s->nloc == s->N;
}

extern "C" int mdqt_observables(mdqt_ctx* s, double out7[7], double* Pvel, double* pops) {
    if (!s) return fail("NULL context");
    if (observables_w1_applies(s)) return observables_w1(s, out7, Pvel, pops, nullptr);
    const int N = s->N;
    double o[5];
    if (mdqt_allgather_positions(s)) return -1;          // collective when sharded
    // pass 1: <vx> (:934-938)
    HIPCHK(hipSetDevice(s->dev));
    HIPCHK(launch_sum_vx(s->dV, s->nloc, s->dScr, s->stream));
    double sumvx = 0.;
    HIPCHK(hipMemcpyAsync(&sumvx, s->dScr, sizeof(double), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    if (s->nloc == 0) sumvx = 0.;
    if (mdqt_allreduce_sum(s, &sumvx, 1)) return -1;
    const double velXAvg = N > 0 ? sumvx / (double)N : 0.;
    std::vector<double> P((size_t)3 * NBINS + 5);
    if (mdqt_partial_observables(s, velXAvg, o, P.data())) return -1;
    memcpy(P.data() + 3 * NBINS, o, sizeof o);
    if (mdqt_allreduce_sum(s, P.data(), P.size())) return -1;
    memcpy(o, P.data() + 3 * NBINS, sizeof o);
    const double EkinX = o[1] / (double)N, EkinY = o[2] / (double)N, EkinZ = o[3] / (double)N;   // :945-947
    s->Epot = (o[4] / 2.) / (double)N;                                                          // :948
    out7[0] = s->t; out7[1] = EkinX; out7[2] = EkinY; out7[3] = EkinZ; out7[4] = s->Epot;
    out7[5] = EkinX + EkinY + EkinZ + s->Epot - s->Epot0; out7[6] = velXAvg;                   // :954
    if (Pvel) {
        const double norm = (6.0 * sqrt(2 * M_PI * 0.002 * 0.002));                            // :975-978
        for (int j = 0; j < 3 * NBINS; ++j) Pvel[j] = P[j] / norm;
    }
    if (pops) {                                                                                 // :1016-1023
        std::vector<double> psi((size_t)24 * N, 0.);
        if (mdqt_get_state(s, nullptr, nullptr, nullptr, N, psi.data(), nullptr, nullptr)) return -1;
        if (mdqt_allreduce_sum(s, psi.data(), psi.size())) return -1;   // zero-padded gather
        for (int i = 0; i < N; i++) {
            const double* w = psi.data() + (size_t)24 * i;
            auto nrm = [&](int k) { return w[2 * k] * w[2 * k] + w[2 * k + 1] * w[2 * k + 1]; };
            pops[3 * i + 0] = nrm(0) + nrm(1);
            if (s->p.qt_model == 3) {                       // 422 pumping: P = 2, 3; D = 4
                pops[3 * i + 1] = nrm(2) + nrm(3);
                pops[3 * i + 2] = nrm(4);
            } else {
                pops[3 * i + 1] = nrm(2) + nrm(3) + nrm(4) + nrm(5);
                pops[3 * i + 2] = nrm(6) + nrm(7) + nrm(8) + nrm(9) + nrm(10) + nrm(11);
            }
        }
    }
    return 0;
}

// ---------------------------------------------------------------------------------------------
// files (reference formats, SpeedUp:725-1032) and the time loop (main, :1139-1383)
// ---------------------------------------------------------------------------------------------

static FILE* open_in(const mdqt_ctx* s, const char* name, const char* mode) {
    char path[1400];
    snprintf(path, sizeof(path), "%s%s", s->saveDirectory, name);
    FILE* f = fopen(path, mode);
    if (!f) fail("cannot open %s: %s", path, strerror(errno));
    return f;
}

extern "C" const char* mdqt_save_directory(const mdqt_ctx* s) { return s->saveDirectory; }

// the reference's "(unsigned)(x)" printed with %d (x86-64 runtime behaviour)
static int ref_udcast(double x) { return (int)(uint32_t)(int64_t)x; }

extern "C" int mdqt_setup_directories(mdqt_ctx* s) {       // SpeedUp:1145-1160
    const mdqt_params* p = &s->p;
    char base[512];
    strncpy(base, p->saveDirectory, sizeof(base) - 1);
    base[sizeof(base) - 1] = 0;
    mkdir(base, 0777);
    char name[256];
    snprintf(name, sizeof name, "Ge%dDensity%dE+11Sig0%dTe%dSigFrac%dDetSP%dDetDP%dOmSP%dOmDP%dNumIons%d",
             ref_udcast(100 * p->Ge), ref_udcast(p->density * 1000), ref_udcast(10 * p->sig0), ref_udcast(p->Te),
             ref_udcast(p->fracOfSig * 100), ref_udcast(p->detuning * 100), ref_udcast(p->detuningDP * 100),
             ref_udcast(p->Om * 100), ref_udcast(p->OmDP * 100), ref_udcast((double)p->N0));
    snprintf(s->saveDirectory, sizeof(s->saveDirectory), "%s%s", base, name);
    mkdir(s->saveDirectory, 0777);
    char jb[64];
    snprintf(jb, sizeof jb, "/job%d/", (int)p->job);
    strncat(s->saveDirectory, jb, sizeof(s->saveDirectory) - strlen(s->saveDirectory) - 1);
    mkdir(s->saveDirectory, 0777);
    struct stat st;
    if (stat(s->saveDirectory, &st) != 0 || !S_ISDIR(st.st_mode))
        return fail("cannot create output directory %s", s->saveDirectory);
    return 0;
}

static FileWriter& writer_of(mdqt_ctx* s) {
    if (!s->writer) s->writer.reset(new FileWriter(4));
    return *s->writer;
}

static std::string path_in(const mdqt_ctx* s, const char* name) { return std::string(s->saveDirectory) + name; }

// wait for the background writers; reports the first file error
static int flush_files(mdqt_ctx* s) {
    if (!s->writer) return 0;
    std::string e;
    if (s->writer->flush(&e)) return fail("%s", e.c_str());
    return 0;
}

// output(), SpeedUp:917-1032.  The observables are computed on the device and snapshotted here;
// the files are formatted by the background writers (the caller flushes: mdqt_output at once,
// mdqt_run at the end of the run).
static int output_async(mdqt_ctx* s) {
    const int N = s->N;
    double o[7];
    auto P = std::make_shared<std::vector<double>>((size_t)3 * NBINS);
    auto pops = std::make_shared<std::vector<double>>((size_t)3 * (N > 0 ? N : 1));
    auto V = std::make_shared<std::vector<double>>((size_t)3 * (N > 0 ? N : 1), 0.);
    if (observables_w1_applies(s)) {                                 // one pass, one synchronisation
        if (observables_w1(s, o, P->data(), pops->data(), V->data())) return -1;
    } else {
        if (mdqt_observables(s, o, P->data(), pops->data())) return -1;
        if (mdqt_get_state(s, nullptr, V->data(), nullptr, N, nullptr, nullptr, nullptr)) return -1;
        if (mdqt_allreduce_sum(s, V->data(), (size_t)N)) return -1;  // vx column, zero-padded gather
    }
    if (s->p.rank != 0) { s->counter++; return 0; }                 // files are rank 0's
    FILE* fa = open_in(s, "energies.dat", "a");                      // appended in order: here
    if (!fa) return -1;
    fprintf(fa, "%lg\t%lg\t%lg\t%lg\t%lg\t%lg\t%lg\n", o[0], o[1], o[2], o[3], o[4], o[5], o[6]);   // :954
    fclose(fa);
    FileWriter& w = writer_of(s);
    const double* vel = s->vel;                                      // constant bin centres
    const char* axes[3] = {"X", "Y", "Z"};
    for (int a = 0; a < 3; ++a) {                                                        // :983-1006
        char b[64];
        snprintf(b, sizeof b, "vel_dist%s_time%06d.dat", axes[a], s->counter);
        const double shift = a == 0 ? o[6] : 0.;
        w.submit(path_in(s, b), "w", [P, vel, a, shift](LgText& t) {
            const double* p = P->data() + (size_t)a * NBINS;
            for (int i = 0; i < NBINS; i++) {
                t.num(vel[i] + shift); t.ch('\t'); t.num(p[i]); t.ch('\n');
            }
        });
    }
    char b[64];
    snprintf(b, sizeof b, "statePopulationsVsVTime%06d.dat", s->counter);
    w.submit(path_in(s, b), "w", [V, pops, N](LgText& t) {                              // :1010-1024
        const double *v = V->data(), *q = pops->data();
        for (int i = 0; i < N; i++) {
            t.num(v[i]); t.ch('\t'); t.num(q[3 * i]); t.ch('\t'); t.num(q[3 * i + 1]); t.ch('\t');
            t.num(q[3 * i + 2]); t.ch('\n');
        }
    });
    s->counter++;                                                                        // :1027
    return 0;
}

extern "C" int mdqt_output(mdqt_ctx* s) {                 // output(), SpeedUp:917-1032
    if (!s) return fail("NULL context");
    if (output_async(s)) return -1;
    return flush_files(s);
}

// writeConditions, SpeedUp:725-784 (files formatted by the background writers)
static int write_conditions_async(mdqt_ctx* s, int c0) {
    const int N = s->N;
    const size_t n1 = (size_t)(N > 0 ? N : 1);
    auto R = std::make_shared<std::vector<double>>(3 * n1, 0.);
    auto V = std::make_shared<std::vector<double>>(3 * n1, 0.);
    auto psi = std::make_shared<std::vector<double>>(24 * n1, 0.);
    if (mdqt_allgather_positions(s)) return -1;           // collective when sharded
    if (mdqt_get_state(s, R->data(), V->data(), nullptr, N, psi->data(), nullptr, nullptr)) return -1;
    if (mdqt_allreduce_sum(s, V->data(), V->size())) return -1;
    if (mdqt_allreduce_sum(s, psi->data(), psi->size())) return -1;
    if (s->p.rank != 0) return 0;
    char b[96];
    snprintf(b, sizeof b, "ions_timestep%06d.dat", c0);
    FILE* fa = open_in(s, b, "w");
    if (!fa) return -1;
    fprintf(fa, "%i\t%i", N, s->counter);                                                // :737
    fclose(fa);
    FileWriter& w = writer_of(s);
    snprintf(b, sizeof b, "conditions_timestep%06d.dat", c0);
    w.submit(path_in(s, b), "w", [R, V, N](LgText& t) {                                 // :747
        const double *r = R->data(), *v = V->data();
        for (int i = 0; i < N; i++) {
            for (int k = 0; k < 3; ++k) { t.num(r[(size_t)k * N + i]); t.ch('\t'); }
            for (int k = 0; k < 3; ++k) { t.num(v[(size_t)k * N + i]); t.ch('\t'); }
            t.ch('\n');
        }
    });
    auto vholder = std::make_shared<std::vector<double>>(s->Vholder);
    for (int v = 0; v < NINTERVALV; v++) {                                              // :752-763
        snprintf(b, sizeof b, "VZERO_timestep%06d_interval%d.dat", c0, v);
        w.submit(path_in(s, b), "w", [vholder, v, N](LgText& t) {
            const double* vh = vholder->data() + (size_t)v * 3 * N;
            for (int i = 0; i < N; i++) {
                t.num(vh[i]); t.ch('\t'); t.num(vh[(size_t)N + i]); t.ch('\t'); t.num(vh[(size_t)2 * N + i]);
                t.ch('\n');
            }
        });
    }
    snprintf(b, sizeof b, "wvFns_timestep%06d.dat", c0);
    w.submit(path_in(s, b), "w", [psi, N](LgText& t) {                                  // :777-779
        for (int j = 0; j < N; j++) {
            const double* ps = psi->data() + (size_t)24 * j;
            for (int k = 0; k < NS; k++) { t.num(ps[2 * k]); t.ch('\t'); t.num(ps[2 * k + 1]); t.ch('\t'); }
            t.ch('\n');
        }
    });
    return 0;
}

extern "C" int mdqt_write_conditions(mdqt_ctx* s, int c0) {   // writeConditions, :725-784
    if (!s) return fail("NULL context");
    if (write_conditions_async(s, c0)) return -1;
    return flush_files(s);
}

extern "C" int mdqt_flush_files(mdqt_ctx* s) {
    if (!s) return fail("NULL context");
    return flush_files(s);
}

extern "C" int mdqt_read_conditions(mdqt_ctx* s, int c0) {    // readConditions, :785-916
    if (!s) return fail("NULL context");
    if (flush_files(s)) return -1;                       // the files may still be being written
    s->t = ((double)c0 - 9.) * TIMESTEP + 0.02;                                         // :789
    char b[96];
    snprintf(b, sizeof b, "ions_timestep%06d.dat", c0);
    FILE* fa = open_in(s, b, "r");
    if (!fa) return -1;
    int j, m, N = -1;
    while (fscanf(fa, "%i\t%i", &j, &m) == 2) { N = j; s->counter = (unsigned)m; }      // :805-814
    fclose(fa);
    if (N < 0) return fail("%s: no ion count", b);
    std::vector<double> R((size_t)3 * (N > 0 ? N : 1), 0.), V(R.size(), 0.), psi((size_t)24 * (N > 0 ? N : 1), 0.);
    snprintf(b, sizeof b, "conditions_timestep%06d.dat", c0);
    fa = open_in(s, b, "r");
    if (!fa) return -1;
    double a, bb, z, d, e, f;
    int i = 0;
    while (i < N && fscanf(fa, "%lg\t%lg\t%lg\t%lg\t%lg\t%lg\n", &a, &bb, &z, &d, &e, &f) == 6) {   // :818-832
        R[i] = a; R[(size_t)N + i] = bb; R[(size_t)2 * N + i] = z;
        V[i] = d; V[(size_t)N + i] = e; V[(size_t)2 * N + i] = f;
        i++;
    }
    fclose(fa);
    if (i != N) return fail("%s: %d of %d rows", b, i, N);
    snprintf(b, sizeof b, "wvFns_timestep%06d.dat", c0);
    fa = open_in(s, b, "r");
    if (!fa) return -1;
    i = 0;
    double w[24];
    while (i < N &&
           fscanf(fa, "%lg%lg\t%lg%lg\t%lg%lg\t%lg%lg\t%lg%lg\t%lg%lg\t%lg%lg\t%lg%lg\t%lg%lg\t%lg%lg\t%lg%lg\t%lg%lg\n",
                  &w[0], &w[1], &w[2], &w[3], &w[4], &w[5], &w[6], &w[7], &w[8], &w[9], &w[10], &w[11], &w[12],
                  &w[13], &w[14], &w[15], &w[16], &w[17], &w[18], &w[19], &w[20], &w[21], &w[22], &w[23]) == 24) {  // :859-894
        memcpy(psi.data() + (size_t)24 * i, w, sizeof(w));
        i++;
    }
    fclose(fa);
    if (i != N) return fail("%s: %d of %d rows", b, i, N);
    const double t = s->t;
    if (resize(s, N)) return -1;
    for (int v = 0; v < NINTERVALV; v++) {                                              // :898-913
        snprintf(b, sizeof b, "VZERO_timestep%06d_interval%d.dat", c0, v);
        fa = open_in(s, b, "r");
        if (!fa) return -1;
        double* vh = s->Vholder.data() + (size_t)v * 3 * N;
        i = 0;
        while (i < N && fscanf(fa, "%lg\t%lg\t%lg", &a, &bb, &z) == 3) {
            vh[i] = a; vh[(size_t)N + i] = bb; vh[(size_t)2 * N + i] = z;
            i++;
        }
        fclose(fa);
    }
    std::vector<double> tp((size_t)(N > 0 ? N : 1), 0.);       // tPart not restored (App. C-8)
    if (upload(s, R.data(), V.data(), N, psi.data(), tp.data())) return -1;
    s->t = t;
    s->c0 = c0;
    s->qidx = (uint64_t)(c0 + 1) * (uint64_t)s->ratio;
    return 0;
}

extern "C" int mdqt_run(mdqt_ctx* s) {                        // main(), SpeedUp:1139-1383
    if (!s) return fail("NULL context");
    if (s->p.world_size > 1 && !s->comm) return fail("mdqt_run: sharded run needs mdqt_comm_init first");
    if (mdqt_setup_directories(s)) return -1;
    if (s->p.newRun == 1) {
        if (mdqt_init(s)) return -1;
    } else {
        s->c0 = s->p.c0;
        if (mdqt_read_conditions(s, s->c0)) return -1;
    }
    const double tend = s->p.tmax + 0.0009;
    const int sf = s->p.sampleFreq, ratio = s->ratio;
    int tsc = ratio;                                                                    // :1235
    while (s->t <= tend) {                                                              // :1248
        if ((s->c0 + 1) % sf == 0 && tsc == 1)                                          // :1365
            if (output_async(s)) return -1;             // files formatted while the loop goes on
        if (tsc == ratio) {                                                             // :1369
            // a whole interval without an output or the end inside it: one k_md_step launch
            if (fused_applies(s)) {
                const long c1 = s->c0 + 1;
                int n = 0, ts = 0;
                double tt = s->t;
                do {
                    n++; ts++; tt += s->dtQ;
                } while (n < MAXSUB && tt <= tend && !((c1 + 1) % sf == 0 && ts == 1) && ts != ratio);
                if (n == ratio) {
                    if (local_reduce(s) || md_step_fused(s)) return -1;
                    s->last_fused = 1;
                    s->c0++;
                    continue;                            // tsc stays = ratio
                }
            }
            s->last_fused = 0;
            if (mdqt_allgather_positions(s)) return -1;                                 // §8e
            if (mdqt_forces(s)) return -1;
            s->c0++;
            tsc = 0;
        }
        // fuse the following iterations while they are pure step();qstep() (App. C-9)
        int n = 0, ts = tsc;
        double tt = s->t;
        do {
            n++; ts++; tt += s->dtQ;
        } while (n < MAXSUB && tt <= tend && !((s->c0 + 1) % sf == 0 && ts == 1) && ts != ratio);
        if (mdqt_substeps(s, n)) return -1;                                            // :1376-1377
        tsc += n;
    }
    return mdqt_write_conditions(s, s->c0);             // :1381; also joins the writers
}

// ---------------------------------------------------------------------------------------------
// The optical-pumping programs' main() — randomFrozenStartTag408Linear.cpp (":" lines below),
// randomFrozenStartTag408Quad.cpp, randomFrozenStartTag422Linear.cpp (same flow).
// ---------------------------------------------------------------------------------------------

static int setup_directories_pump(mdqt_ctx* s) {                // :985-999
    const mdqt_params* p = &s->p;
    char base[512];
    strncpy(base, p->saveDirectory, sizeof(base) - 1);
    base[sizeof(base) - 1] = 0;
    mkdir(base, 0777);
    char name[256];
    snprintf(name, sizeof name, "PumpTime%dPumpStart%dDet%dOm%dDensity%dGe%dNumIons%d",
             (int)(unsigned)(1000000000. * p->tpumpreal), (int)(unsigned)(p->tstartV0),
             (int)(unsigned)(100. * fabs(p->detuning)), (int)(unsigned)(100. * p->Om),
             (int)(unsigned)(10. * p->density), (int)(unsigned)(1000 * p->Ge), (int)(unsigned)p->N0);
    snprintf(s->saveDirectory, sizeof(s->saveDirectory), "%s%s", base, name);
    mkdir(s->saveDirectory, 0777);
    char jb[64];
    snprintf(jb, sizeof jb, "/job%d/", (int)p->job);
    strncat(s->saveDirectory, jb, sizeof(s->saveDirectory) - strlen(s->saveDirectory) - 1);
    mkdir(s->saveDirectory, 0777);
    struct stat st;
    if (stat(s->saveDirectory, &st) != 0 || !S_ISDIR(st.st_mode))
        return fail("cannot create output directory %s", s->saveDirectory);
    return 0;
}

// step() :377-394: step_R(dt/2) (at t == 0 with forces() first and the DT^2 F term), step_V(dt)
// with forces() at the half-drifted positions, step_R(dt/2)
static int md_step_pump(mdqt_ctx* s) {
    const double dt = s->dtQ * s->ratio;                         // :389 dt=quantumTimestep*ratio
    const double DT = 0.5 * dt, DT2 = DT * DT;
    const int moving = s->t > 0 ? 1 : 0;
    HIPCHK(hipSetDevice(s->dev));
    double* R = s->dR;
    if (!moving) {                                               // :331 forces() before the first drift
        if (mdqt_forces(s)) return -1;
        if (settle_forces(s)) return -1;
    }
    HIPCHK(launch_leapfrog_half(R, s->dV, s->dF, s->nloc, s->S, s->L, DT, DT2, moving, 0., s->stream));
    if (mdqt_forces(s)) return -1;                               // step_V: forces() :361
    if (settle_forces(s)) return -1;
    HIPCHK(launch_leapfrog_half(R, s->dV, s->dF, s->nloc, s->S, s->L, DT, DT2, moving, dt, s->stream));
    return 0;
}

// measureSpinUps() :600-665 (tags from the Philox stream, mdqt_tag_spin_up)
static int measure_spin_ups(mdqt_ctx* s) {
    const int N = s->N;
    s->spinUp.assign((size_t)(N > 0 ? N : 1), 0);
    int n_up = 0;
    if (mdqt_tag_spin_up(s, s->spinUp.data(), &n_up)) return -1;
    s->nSpinUp = n_up;
    if (!s->dSpinUp) HIPCHK(hipMalloc(&s->dSpinUp, (size_t)s->capS * sizeof(int)));
    HIPCHK(hipMemcpyAsync(s->dSpinUp, s->spinUp.data(), (size_t)N * sizeof(int), hipMemcpyHostToDevice, s->stream));
    char b[96];
    snprintf(b, sizeof b, "spinUpIons_timestep%06d.dat", s->c0);
    FILE* fa = open_in(s, b, "w");
    if (!fa) return -1;
    fprintf(fa, "%i", s->nSpinUp);                               // :651-662
    fclose(fa);
    return 0;
}

// output() :799-935: energies (EkinX without subtracting <vx>), the spin-up ions' moments and x
// velocity distribution over 4001 bins, counter++; host sums in the reference's order
static int output_pump(mdqt_ctx* s) {
    const int N = s->N;
    std::vector<double> V((size_t)3 * (N > 0 ? N : 1), 0.);
    if (mdqt_get_state(s, nullptr, V.data(), nullptr, N, nullptr, nullptr, nullptr)) return -1;
    double EkinX = 0., EkinY = 0., EkinZ = 0.;
    for (int i = 0; i < N; i++) {                                // :812-817
        EkinX += 0.5 * (V[i] * V[i]);
        EkinY += 0.5 * (V[(size_t)N + i] * V[(size_t)N + i]);
        EkinZ += 0.5 * (V[(size_t)2 * N + i] * V[(size_t)2 * N + i]);
    }
    EkinX /= (double)N; EkinY /= (double)N; EkinZ /= (double)N;
    double e;
    if (mdqt_epotential(s, &e)) return -1;                       // :821
    FILE* fa = open_in(s, "energies.dat", "a");                  // :825-829
    if (!fa) return -1;
    fprintf(fa, "%lg\t%lg\t%lg\t%lg\t%lg\t%lg\n", s->t, EkinX, EkinY, EkinZ, s->Epot,
            EkinX + EkinY + EkinZ + s->Epot - s->Epot0);
    fclose(fa);
    // tagged x distribution on the device (:831-864 exp(-V2 (vel_j - v)^2) summed over spin-up ions)
    const int nch = (N + 255) / 256;
    if (!s->dTkde) HIPCHK(hipMalloc(&s->dTkde, ((size_t)(nch > 0 ? nch : 1) + 1) * 3 * TKDE_BINS * sizeof(double)));
    if (!s->dSpinUp) {
        HIPCHK(hipMalloc(&s->dSpinUp, (size_t)s->capS * sizeof(int)));
        HIPCHK(hipMemsetAsync(s->dSpinUp, 0, (size_t)s->capS * sizeof(int), s->stream));
    }
    std::vector<double> P((size_t)3 * TKDE_BINS, 0.);
    if (N > 0) {
        HIPCHK(launch_tagged_kde(s->dV, s->dSpinUp, N, s->S, s->dTkde + (size_t)3 * TKDE_BINS, s->dTkde, s->stream,
                                 s->pumpBin0));
        HIPCHK(hipMemcpyAsync(P.data(), s->dTkde, P.size() * sizeof(double), hipMemcpyDeviceToHost, s->stream));
        HIPCHK(hipStreamSynchronize(s->stream));
    }
    // moments of the tagged x velocities (:836-851, :866-876)
    double m1 = 0, m2 = 0, m3 = 0, m4 = 0;
    unsigned nt = 0;
    const bool have = !s->spinUp.empty() && (int)s->spinUp.size() >= N;
    for (int i = 0; i < N; i++) {
        const double v = V[i];
        if (have && s->spinUp[i]) {
            m1 += v; m2 += v * v; m3 += v * v * v; m4 += v * v * v * v;
            nt += 1;
        }
    }
    m1 /= nt; m2 /= nt; m3 /= nt; m4 /= nt;
    fa = open_in(s, "taggedMoments.dat", "a");
    if (!fa) return -1;
    fprintf(fa, "%lg\t%lg\t%lg\t%lg\t%lg\n", s->t, m1, m2, m3, m4);
    fclose(fa);
    char b[96];
    snprintf(b, sizeof b, "vel_distX_timestep%06d.dat", s->c0);   // :887-901 (X only)
    fa = open_in(s, b, "w");
    if (!fa) return -1;
    for (int j = 0; j < TKDE_BINS; j++) fprintf(fa, "%lg\t%lg\n", (double)(j + s->pumpBin0) * 0.0025, P[j]);
    fclose(fa);
    s->counter++;                                                // :929
    return 0;
}

// Zfunc(c1V) + printVAF(t) :938-975 (host, the reference's order)
static int vaf_pump(mdqt_ctx* s, int c1V) {
    const int N = s->N;
    std::vector<double> V((size_t)3 * (N > 0 ? N : 1), 0.);
    if (mdqt_get_state(s, nullptr, V.data(), nullptr, N, nullptr, nullptr, nullptr)) return -1;
    if (c1V == 0) s->vaHold.assign(V.begin(), V.begin() + N);
    if ((int)s->vaHold.size() < N) s->vaHold.resize((size_t)N, 0.);
    double VAF = 0.0;
    for (int j = 0; j < N; j++) VAF += 1 / ((double)(N)) * (s->vaHold[j] * V[j]);
    FILE* fa = open_in(s, "VAF.dat", "a");
    if (!fa) return -1;
    fprintf(fa, "%lg\t%lg\n", s->t, VAF);
    fclose(fa);
    return 0;
}

static int write_conditions_pump(mdqt_ctx* s, int c0) {        // :667-707
    const int N = s->N;
    std::vector<double> R((size_t)3 * (N > 0 ? N : 1), 0.), V(R.size(), 0.);
    if (mdqt_get_state(s, R.data(), V.data(), nullptr, N, nullptr, nullptr, nullptr)) return -1;
    char b[96];
    snprintf(b, sizeof b, "ions_timestep%06d.dat", c0);
    FILE* fa = open_in(s, b, "w");
    if (!fa) return -1;
    fprintf(fa, "%i\t%i", N, s->counter);
    fclose(fa);
    snprintf(b, sizeof b, "spinUpIonsList_timestep%06d.dat", c0);
    fa = open_in(s, b, "w");
    if (!fa) return -1;
    for (int i = 0; i < N; i++) fprintf(fa, "%i\n", (int)s->spinUp.size() > i ? s->spinUp[i] : 0);
    fclose(fa);
    snprintf(b, sizeof b, "conditions_timestep%06d.dat", c0);
    fa = open_in(s, b, "w");
    if (!fa) return -1;
    for (int i = 0; i < N; i++)
        fprintf(fa, "%lg\t%lg\t%lg\t%lg\t%lg\t%lg\t\n", R[i], R[(size_t)N + i], R[(size_t)2 * N + i], V[i],
                V[(size_t)N + i], V[(size_t)2 * N + i]);
    fclose(fa);
    return 0;
}

static int read_conditions_pump(mdqt_ctx* s, int c0) {         // :709-797
    s->t = ((double)c0 - 9.) * TIMESTEP + 0.02;                 // :713
    s->pumpBin0 = 0;                                             // :721-724 vel[i] = i 0.0025
    char b[96];
    snprintf(b, sizeof b, "ions_timestep%06d.dat", c0);
    FILE* fa = open_in(s, b, "r");
    if (!fa) return -1;
    int j, m, N = -1;
    while (fscanf(fa, "%i\t%i", &j, &m) == 2) { N = j; s->counter = (unsigned)m; }
    fclose(fa);
    if (N < 0) return fail("%s: no ion count", b);
    std::vector<int> up((size_t)(N > 0 ? N : 1), 0);
    snprintf(b, sizeof b, "spinUpIonsList_timestep%06d.dat", c0);
    fa = open_in(s, b, "r");
    if (!fa) return -1;
    int i = 0, sUp;
    while (i < N && fscanf(fa, "%i\n", &sUp) == 1) up[i++] = sUp;
    fclose(fa);
    std::vector<double> R((size_t)3 * (N > 0 ? N : 1), 0.), V(R.size(), 0.);
    snprintf(b, sizeof b, "conditions_timestep%06d.dat", c0);
    fa = open_in(s, b, "r");
    if (!fa) return -1;
    double a, bb, z, d, e, f;
    i = 0;
    while (i < N && fscanf(fa, "%lg\t%lg\t%lg\t%lg\t%lg\t%lg\n", &a, &bb, &z, &d, &e, &f) == 6) {
        R[i] = a; R[(size_t)N + i] = bb; R[(size_t)2 * N + i] = z;
        V[i] = d; V[(size_t)N + i] = e; V[(size_t)2 * N + i] = f;
        i++;
    }
    fclose(fa);
    if (i != N) return fail("%s: %d of %d rows", b, i, N);
    const double t = s->t;
    if (resize(s, N)) return -1;
    // wvFns are not read (the reference's read loop is commented out, :772-795): they stay zero
    std::vector<double> psi((size_t)24 * (N > 0 ? N : 1), 0.), tp((size_t)(N > 0 ? N : 1), 0.);
    if (upload(s, R.data(), V.data(), N, psi.data(), tp.data())) return -1;
    s->spinUp = up;
    s->nSpinUp = 0;
    for (int k = 0; k < N; ++k) s->nSpinUp += up[k] ? 1 : 0;
    if (s->dSpinUp) { (void)hipFree(s->dSpinUp); s->dSpinUp = nullptr; }
    HIPCHK(hipMalloc(&s->dSpinUp, (size_t)s->capS * sizeof(int)));
    HIPCHK(hipMemcpyAsync(s->dSpinUp, up.data(), (size_t)N * sizeof(int), hipMemcpyHostToDevice, s->stream));
    s->t = t;
    s->c0 = c0;
    return 0;
}

extern "C" int mdqt_get_spin_up_list(mdqt_ctx* s, int* tags, int* n_up) {
    if (!s) return fail("NULL context");
    for (int i = 0; i < s->N && tags; ++i) tags[i] = (int)s->spinUp.size() > i ? s->spinUp[i] : 0;
    if (n_up) *n_up = s->nSpinUp;
    return 0;
}

extern "C" int mdqt_run_pump(mdqt_ctx* s) {                     // main() :981-1076
    if (!s) return fail("NULL context");
    if (s->p.qt_model < 1 || s->p.qt_model > 3) return fail("mdqt_run_pump: qt_model must be 1, 2 or 3");
    if (s->p.world_size != 1) return fail("mdqt_run_pump: world_size 1 only");
    if (setup_directories_pump(s)) return -1;
    int recorded = 0;                                            // recordedSpinUps :81
    s->spinUp.clear();
    s->nSpinUp = 0;
    s->pumpBin0 = -2000;
    if (s->p.newRun == 1) {                                      // :1036-1046
        if (mdqt_init(s)) return -1;
    } else {
        if (read_conditions_pump(s, s->p.c0)) return -1;
        recorded = 1;
    }
    const double tpump = s->p.tpumpreal * 813490 * sqrt(s->p.density);      // :79
    const double tendV0 = s->p.tstartV0 + tpump;                             // :80
    const double tstartV0 = s->p.tstartV0;
    const double tend = s->p.tmax + 0.0009;
    const int sf = s->p.sampleFreq, ratio = s->ratio;
    int tsc = ratio;                                             // :1033
    // quantum steps are queued while nothing else happens and run as one fused launch
    int pending = 0;
    double tv = s->t;                                            // the loop's t (s->t lags by `pending` qsteps)
    auto flush = [&]() -> int {
        if (pending > 0) {
            if (run_substeps(s, pending, 0, 1, 1)) return -1;    // qstep() x pending :396-598
            pending = 0;
            if (s->t != tv) return fail("mdqt_run_pump: time bookkeeping mismatch");
        }
        return 0;
    };
    while (tv <= tend) {                                         // :1050
        if (recorded == 0 && tv >= tendV0) {                     // :1052-1058
            if (flush()) return -1;
            if (measure_spin_ups(s)) return -1;
            recorded = 1;
            if (output_pump(s)) return -1;
            if (vaf_pump(s, 0)) return -1;
        }
        if ((s->c0 + 1) % sf == 0 && tsc == 1 && recorded == 1) {   // :1062-1069
            if (flush()) return -1;
            if (output_pump(s)) return -1;
            if (vaf_pump(s, 1)) return -1;
        }
        if (tsc == ratio) {                                      // :1070-1074
            if (flush()) return -1;
            if (md_step_pump(s)) return -1;
            s->c0++;
            tsc = 0;
        }
        if (tv < tendV0 && tv > tstartV0) {                      // :1075-1077 qstep()
            pending++;
            tv += s->dtQ;                                        // qstep's t += dtQuant :597
            if (pending == MAXSUB && flush()) return -1;
        } else {                                                 // :1078-1080
            if (flush()) return -1;
            s->t += s->dtQ;
            tv = s->t;
        }
        tsc++;
    }
    if (flush()) return -1;
    if (flush_files(s)) return -1;
    return write_conditions_pump(s, s->c0);                      // :1084
}

// ---------------------------------------------------------------------------------------------
// streams, timing, multi-GPU plumbing
// ---------------------------------------------------------------------------------------------

extern "C" int mdqt_set_option(mdqt_ctx* s, const char* name, int value) {
    if (!s || !name) return fail("mdqt_set_option: NULL argument");
    if (!strcmp(name, "force_scheme")) {
        if (value < 0 || value > 3)
            return fail("force_scheme must be 0 (auto), 1 (rows), 2 (Newton-3 tiles) or 3 (Newton-3 blocks)");
        if (value == 2 && s->p.world_size != 1) return fail("force_scheme 2 needs world_size 1");
        if (settle_forces(s)) return -1;
        s->scheme_opt = value;
        choose_segments(s);
        return ensure_aux(s);
    }
    if (!strcmp(name, "expt_force_sig")) {             // diagnostic: unfused force launches with the fused
        if (value < 0 || value > 1) return fail("expt_force_sig must be 0 or 1");   // step's signalling
        if (value && arrive_setup(s)) return -1;
        s->force_arrive = value ? s->dArrive : nullptr;
        return 0;
    }
    if (!strcmp(name, "potential_n3")) {               // Epotential on the Newton-3 tiles (1) or the rows (0)
        if (value < 0 || value > 1) return fail("potential_n3 must be 0 or 1");
        s->n3_potential = value;
        return 0;
    }
    if (!strcmp(name, "force_n3b_pairs")) {            // Newton-3 blocks: 4 waves on two I tiles each (1) or 8 waves (0)
        if (value < 0 || value > 1) return fail("force_n3b_pairs must be 0 (8 waves, one I tile each) or 1 (4 waves, two each)");
        if (settle_forces(s)) return -1;
        s->n3b_pairs = value;
        return 0;
    }
    if (!strcmp(name, "potential_plan")) {             // Epotential on the blocks: the force call's plan (1) or exact (0)
        if (value < 0 || value > 1) return fail("potential_plan must be 0 (every pair to L/2) or 1 (the plan)");
        s->pot_plan = value;
        return 0;
    }
    if (!strcmp(name, "qt_im01")) {                    // 0: the general FAST lane instance (tests)
        if (value < 0 || value > 1) return fail("qt_im01 must be 0 or 1");
        if (value) {                                   // only where the table allows it
            int ok = 1;
            for (int k = 0; k < 16; ++k)
                if (s->ftab.cre[0][k] != 0. || s->ftab.cre[1][k] != 0.) ok = 0;
            if (!ok) return fail("qt_im01: the static coupling slots are not purely imaginary");
        }
        s->qc.im01 = value;
        return 0;
    }
    if (!strcmp(name, "fused_step")) {                 // one k_md_step launch per MD step (mdqt_md_steps)
        if (value < 0 || value > 1) return fail("fused_step must be 0 or 1");
        s->fused_opt = value;
        return 0;
    }
    if (!strcmp(name, "overlap")) {                    // force || QT launches of an MD step (mdqt_md_steps)
        if (value < 0 || value > 1) return fail("overlap must be 0 or 1");
        s->overlap_opt = value;
        return 0;
    }
    if (!strcmp(name, "force_ufar_exp")) {             // ultra-far pair form: eps = 10^-value (0: off)
        if (value < 0 || value > 300) return fail("force_ufar_exp must be 0 (off) .. 300");
        // (force_form_mode 1: the measured sums hold its terms — forget what earlier calls measured)
        if (value != s->ufar_exp && form_measured(s) && (settle_forces(s) || tail_reset(s))) return -1;
        s->ufar_exp = value;
        return 0;
    }
    if (!strcmp(name, "force_vfar_exp")) {             // very-far pair form: eps = 10^-value (0: off)
        if (value < 0 || value > 300) return fail("force_vfar_exp must be 0 (off) .. 300");
        // (force_form_mode 1: the measured sums hold its terms — forget what earlier calls measured)
        if (value != s->vfar_exp && form_measured(s) && (settle_forces(s) || tail_reset(s))) return -1;
        s->vfar_exp = value;
        return 0;
    }
    if (!strcmp(name, "force_mid_exp")) {              // mid pair form: eps = 10^-value (0: off)
        if (value < 0 || value > 300) return fail("force_mid_exp must be 0 (off) .. 300");
        // (force_form_mode 1: the measured sums hold its terms — forget what earlier calls measured)
        if (value != s->mid_exp && form_measured(s) && (settle_forces(s) || tail_reset(s))) return -1;
        s->mid_exp = value;
        return 0;
    }
    if (!strcmp(name, "force_far_exp")) {              // far pair form: eps = 10^-value (0: off)
        if (value < 0 || value > 300) return fail("force_far_exp must be 0 (off) .. 300");
        // (force_form_mode 1: the measured sums hold its terms — forget what earlier calls measured)
        if (value != s->far_exp && form_measured(s) && (settle_forces(s) || tail_reset(s))) return -1;
        s->far_exp = value;
        return 0;
    }
    if (!strcmp(name, "force_tail_exp")) {             // error-bounded tail: eps = 10^-value (0: exact)
        if (value < 0 || value > 300) return fail("force_tail_exp must be 0 (exact) .. 300");
        if (value != s->tail_exp && (settle_forces(s) || tail_reset(s))) return -1;
        s->tail_exp = value;
        return 0;
    }
    if (!strcmp(name, "force_form_mode")) {            // the tiers' radii: 0 a priori, 1 measured and enforced
        if (value < 0 || value > 2)
            return fail("force_form_mode must be 0 (a priori), 1 (measured) or 2 (measured, sharing an exact tail's eps)");
        if (value != s->form_mode && (settle_forces(s) || tail_reset(s))) return -1;
        s->form_mode = value;
        return 0;
    }
    if (!strcmp(name, "force_tail_mode")) {            // 0: a-priori bound, 1: measured and enforced
        if (value < 0 || value > 1) return fail("force_tail_mode must be 0 (a priori) or 1 (measured)");
        if (value != s->tail_mode && (settle_forces(s) || tail_reset(s))) return -1;
        s->tail_mode = value;
        return 0;
    }
    if (!strcmp(name, "force_balance")) {              // sharded Newton-3 blocks: ranges by work (1) or by count (0)
        if (value < 0 || value > 1) return fail("force_balance must be 0 (equal block counts) or 1 (by work)");
        if (value != s->balance_opt) {
            if (settle_forces(s)) return -1;
            s->balance_opt = value;
            if (s->use_n3b) {                           // back to the equal ranges; weighted again at the next call
                const int W = s->p.world_size;
                n3b_set_range(s->n3b, (int)((long)s->p.rank * s->n3b.NB / W), (int)((long)(s->p.rank + 1) * s->n3b.NB / W));
                s->balanced = false;
                if (ensure_aux(s)) return -1;
            }
        }
        return 0;
    }
    if (!strcmp(name, "force_tile_split")) {           // Newton-3 tiles: the last round's whole tile pairs as halves
        if (value < 0 || value > 2) return fail("force_tile_split must be 0 (off), 1 (halves) or 2 (quarters)");
        if (settle_forces(s)) return -1;
        s->split_opt = value;
        return ensure_aux(s);
    }
    if (!strcmp(name, "force_split_cus")) {            // the CU count the split table is cut for (0: the device's)
        if (value < 0 || value > 65536) return fail("force_split_cus must be 0 (the device's CU count) or a CU count");
        if (settle_forces(s)) return -1;
        s->split_cus = value;
        return ensure_aux(s);
    }
    if (!strcmp(name, "force_reduce_mask")) {          // Newton-3 blocks: the reduction reads only written j-slots
        if (value < 0 || value > 1) return fail("force_reduce_mask must be 0 (every j-slot) or 1 (the written ones)");
        if (settle_forces(s)) return -1;
        s->tmask_mode = value;
        return 0;
    }
    if (!strcmp(name, "force_ax1")) {                  // Newton-3 blocks: the one-axis per-pair image instance
        if (value < 0 || value > 1) return fail("force_ax1 must be 0 (off) or 1 (where the skip radius reaches L/2)");
        if (settle_forces(s)) return -1;
        s->ax1_mode = value;
        return 0;
    }
    if (!strcmp(name, "force_sort")) {                 // Newton-3 blocks: Hilbert order + tile-pair skipping
        if (value < 0 || value > 2) return fail("force_sort must be 0 (off), 1 (on) or 2 (sorted, no skipping)");
        if (settle_forces(s)) return -1;
        s->sort_mode = value;
        return ensure_aux(s);
    }
    if (!strcmp(name, "qt_enabled")) {                 // pump window of the tagging programs
        if (value < 0 || value > 1) return fail("qt_enabled must be 0 or 1");
        s->p.qt_enabled = value;
        return 0;
    }
    if (!strcmp(name, "qt_math")) {
        if (value < 0 || value > 2) return fail("qt_math must be 0 (exact), 1 (FMA-contracted) or 2 (reassociated)");
        if (value != 2 && s->p.qt_model != 0) return fail("the optical-pumping qt_models need qt_math 2");
        s->qt_math = value;
        return 0;
    }
    if (!strcmp(name, "force_kernel")) {
        if (value < 0 || value > 1) return fail("force_kernel must be 0 (exact) or 1 (fast)");
        if (value != s->force_variant && (settle_forces(s) || tail_reset(s))) return -1;   // tail_measured changes
        s->force_variant = value;
        return 0;
    }
    if (!strcmp(name, "init_threads")) {                // init() sampling: 0 auto, 1 sequential, k threads
        if (value < 0 || value > 256) return fail("init_threads must be in [0, 256]");
        s->init_threads = value;
        return 0;
    }
    if (!strcmp(name, "substep_kernel")) {
        if (value < 0 || value > 2) return fail("substep_kernel must be 0 (auto), 1 (thread/ion) or 2 (lanes/ion)");
        s->substep_mode = value;
        return 0;
    }
    return fail("unknown option %s", name);
}

extern "C" int mdqt_set_stream(mdqt_ctx* s, void* st) {
    s->stream = st ? (hipStream_t)st : s->own;
    return 0;
}
extern "C" void* mdqt_get_stream(mdqt_ctx* s) { return (void*)s->stream; }
extern "C" int mdqt_synchronize(mdqt_ctx* s) {
    HIPCHK(hipSetDevice(s->dev));
    HIPCHK(hipStreamSynchronize(s->stream));
    return check_range_flag(s);
}
extern "C" int mdqt_positions_device(mdqt_ctx* s, void** dptr, int* S) {
    if (dptr) *dptr = (void*)s->dR;
    if (S) *S = s->S;
    return 0;
}
extern "C" int mdqt_enable_timing_at(mdqt_ctx* s, int on, int kinds, int offset) {
    if (!s) return fail("NULL context");
    if (kinds < 1 || kinds > 15) return fail("mdqt_enable_timing_at: kinds must be 1 .. 15 (bits: force, substeps, potential block kernel, force breakdown)");
    if (on > 0 && (offset < 0 || offset >= on)) return fail("mdqt_enable_timing_at: offset must be in [0, period)");
    s->timing = on > 0;
    s->tperiod = on > 0 ? (unsigned)on : 1u;
    s->toffset = on > 0 ? (unsigned)offset : 0u;
    s->tkinds = (unsigned)kinds;
    s->tcount[0] = s->tcount[1] = 0;
    s->evused[0] = s->evused[1] = s->evused[2] = s->evused[3] = 0;
    for (auto& c : s->bdcalls) {                    // (the breakdown restarts with the timing)
        for (hipEvent_t e : c.m) if (e) s->bdfree.push_back(e);
        if (c.ag0) s->bdfree.push_back(c.ag0);
        if (c.ag1) s->bdfree.push_back(c.ag1);
    }
    s->bdcalls.clear();
    return 0;
}
extern "C" int mdqt_enable_timing_kinds(mdqt_ctx* s, int on, int kinds) {
    return mdqt_enable_timing_at(s, on, kinds, on > 0 ? on / 2 : 0);
}
extern "C" int mdqt_enable_timing(mdqt_ctx* s, int on) { return mdqt_enable_timing_kinds(s, on, 3); }

extern "C" int mdqt_kernel_times(mdqt_ctx* s, double* out, int n) {
    if (!s || !out) return fail("mdqt_kernel_times: NULL argument");
    if (n < 6) return fail("mdqt_kernel_times: need 6 doubles");
    HIPCHK(hipSetDevice(s->dev));
    HIPCHK(hipStreamSynchronize(s->stream));
    for (int k = 0; k < 4; ++k) {
        if (2 * k + 1 >= n) { s->evused[k] = 0; continue; }
        double tot = 0.;
        for (int i = 0; i + 1 < s->evused[k]; i += 2) {
            float ms = 0.f;
            HIPCHK(hipEventElapsedTime(&ms, s->evpool[k][i], s->evpool[k][i + 1]));
            tot += ms;
        }
        out[2 * k] = tot;
        out[2 * k + 1] = (double)(s->evused[k] / 2);
        s->evused[k] = 0;
    }
    return 0;
}

extern "C" int mdqt_kernel_time_totals(mdqt_ctx* s, double* force_ms, int* nforce, double* sub_ms, int* nsub) {
    if (!s) return fail("NULL context");
    double t[6];
    if (mdqt_kernel_times(s, t, 6)) return -1;
    if (force_ms) *force_ms = t[0];
    if (nforce) *nforce = (int)t[1];
    if (sub_ms) *sub_ms = t[2];
    if (nsub) *nsub = (int)t[3];
    return 0;
}

// ---------------------------------------------------------------------------------------------
// RCCL: one communicator per context over world_size ranks (one process per GPU).  Data-path
// collectives per MD step: the all-gather of the position slabs and, for Newton-3
// block pairs (N > 65,536), the reduce-scatter of the per-rank dense partial forces; output
// steps all-reduce a few scalars, the KDE bins and the per-ion file columns.
// ---------------------------------------------------------------------------------------------


extern "C" int mdqt_comm_unique_id(void* out, size_t len) {
    if (!out || len < sizeof(ncclUniqueId)) return fail("mdqt_comm_unique_id: need %zu bytes", sizeof(ncclUniqueId));
    ncclUniqueId id;
    NCCLCHK(ncclGetUniqueId(&id));
    memcpy(out, &id, sizeof id);
    return 0;
}

extern "C" int mdqt_comm_init(mdqt_ctx* s, const void* uid, size_t len) {
    if (!s || !uid || len < sizeof(ncclUniqueId)) return fail("mdqt_comm_init: bad arguments");
    if (s->comm) return fail("mdqt_comm_init: communicator already initialised");
    ncclUniqueId id;
    memcpy(&id, uid, sizeof id);
    HIPCHK(hipSetDevice(s->dev));
    NCCLCHK(ncclCommInitRank(&s->comm, s->p.world_size, id, s->p.rank));
    return 0;
}

extern "C" int mdqt_comm_size(const mdqt_ctx* s, int* n) {
    if (!s || !n) return fail("mdqt_comm_size: bad arguments");
    if (s->comm) {
        NCCLCHK(ncclCommCount(s->comm, n));
    } else {
        *n = s->local.empty() ? 1 : (int)s->local.size();
    }
    return 0;
}

extern "C" int mdqt_comm_init_local(mdqt_ctx* const* ctxs, int n) {
    if (!ctxs || n < 1) return fail("mdqt_comm_init_local: bad arguments");
    for (int r = 0; r < n; ++r) {
        if (!ctxs[r] || ctxs[r]->p.world_size != n || ctxs[r]->p.rank != r)
            return fail("mdqt_comm_init_local: context %d is not rank %d of %d", r, r, n);
        if (ctxs[r]->S != ctxs[0]->S || ctxs[r]->N != ctxs[0]->N)
            return fail("mdqt_comm_init_local: contexts disagree on N");
    }
    for (int r = 0; r < n; ++r) ctxs[r]->local.assign(ctxs, ctxs + n);
    return 0;
}

extern "C" int mdqt_allgather_positions(mdqt_ctx* s) {
    if (!s) return fail("NULL context");
    if (s->p.world_size == 1) return 0;
    const size_t cnt = (size_t)3 * s->S;
    if (!s->comm && !s->local.empty()) {
        // in-process group: push this rank's slab into every peer (callers run the ranks in
        // lockstep: every rank pushes before any rank computes forces)
        HIPCHK(hipSetDevice(s->dev));
        HIPCHK(hipStreamSynchronize(s->stream));
        for (mdqt_ctx* q : s->local) {
            if (q == s) continue;
            // on the PEER's stream: ordered before the peer's next force launch (a plain
            // hipMemcpyPeer is asynchronous for device-to-device copies and races with it)
            HIPCHK(hipMemcpyPeerAsync(q->dR + (size_t)s->p.rank * cnt, q->dev, s->dR + (size_t)s->p.rank * cnt,
                                      s->dev, cnt * sizeof(double), q->stream));
        }
        return 0;
    }
    if (!s->comm) return fail("mdqt_allgather_positions: no communicator (mdqt_comm_init)");
    HIPCHK(hipSetDevice(s->dev));
    const bool bd = force_timed_next(s) && s->use_n3b;   // (the breakdown's first stage)
    for (hipEvent_t& e : s->bd_ag)
        if (e) { s->bdfree.push_back(e); e = nullptr; }
    if (bd) s->bd_ag[0] = bd_event(s);
    NCCLCHK(ncclAllGather(s->dR + (size_t)s->p.rank * cnt, s->dR, cnt, ncclDouble, s->comm, s->stream));
    if (bd) s->bd_ag[1] = bd_event(s);
    return 0;
}

// the force-call breakdown (timing kind bit 3) since the last call: average ms per timed block-scheme force
// call of out[0] the preceding position all-gather (0 at world 1), [1] sort and boxes (with the first sharded
// call's balance census), [2] plan, [3] block kernel (launch to end, incl. its dispatch gap), [4] slot reduction,
// [5] tail pass (all-reduce of the per-sub-tile sums, list, exact fix), [6] reduce-scatter, [7] forces() start to
// end (= [1] + ... + [6]), out[8] the calls; resets
extern "C" int mdqt_force_breakdown(mdqt_ctx* s, double* out, int n) {
    if (!s || !out) return fail("mdqt_force_breakdown: NULL argument");
    if (n < 9) return fail("mdqt_force_breakdown: need 9 doubles");
    HIPCHK(hipSetDevice(s->dev));
    HIPCHK(hipStreamSynchronize(s->stream));
    double acc[8] = {0., 0., 0., 0., 0., 0., 0., 0.};
    auto ms = [](hipEvent_t a, hipEvent_t b) -> double {
        float t = 0.f;
        return (a && b && hipEventElapsedTime(&t, a, b) == hipSuccess) ? (double)t : 0.;
    };
    for (auto& c : s->bdcalls) {
        acc[0] += ms(c.ag0, c.ag1);
        for (int k = 0; k < 6; ++k) acc[1 + k] += ms(c.m[k], c.m[k + 1]);
        acc[7] += ms(c.m[0], c.m[6]);
        for (hipEvent_t e : c.m) if (e) s->bdfree.push_back(e);
        if (c.ag0) s->bdfree.push_back(c.ag0);
        if (c.ag1) s->bdfree.push_back(c.ag1);
    }
    const double nc = (double)s->bdcalls.size();
    for (int k = 0; k < 8; ++k) out[k] = nc > 0 ? acc[k] / nc : 0.;
    out[8] = nc;
    s->bdcalls.clear();
    return 0;
}

extern "C" int mdqt_allreduce_sum(mdqt_ctx* s, double* buf, size_t n) {
    if (!s || (!buf && n)) return fail("mdqt_allreduce_sum: bad arguments");
    if (s->p.world_size == 1 || n == 0) return 0;
    if (!s->comm) return fail("mdqt_allreduce_sum: no communicator (mdqt_comm_init)");
    HIPCHK(hipSetDevice(s->dev));
    if (n > s->dCommCap) {
        if (s->dComm) HIPCHK(hipFree(s->dComm));
        s->dComm = nullptr;
        HIPCHK(hipMalloc(&s->dComm, n * sizeof(double)));
        s->dCommCap = n;
    }
    HIPCHK(hipMemcpyAsync(s->dComm, buf, n * sizeof(double), hipMemcpyHostToDevice, s->stream));
    NCCLCHK(ncclAllReduce(s->dComm, s->dComm, n, ncclDouble, ncclSum, s->comm, s->stream));
    HIPCHK(hipMemcpyAsync(buf, s->dComm, n * sizeof(double), hipMemcpyDeviceToHost, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    return 0;
}

extern "C" int mdqt_slab_bounds(const mdqt_ctx* s, int* lo, int* hi) {
    if (lo) *lo = s->lo;
    if (hi) *hi = s->hi;
    return 0;
}

extern "C" int mdqt_set_counters(mdqt_ctx* s, int c0, unsigned counter, double Epot, double Epot0) {
    s->c0 = c0; s->counter = counter; s->Epot = Epot; s->Epot0 = Epot0;
    return 0;
}

extern "C" int mdqt_get_drand48_state(mdqt_ctx* s, uint64_t* x) {
    if (!s || !x) return fail("mdqt_get_drand48_state: bad arguments");
    if (!s->dX48) { *x = s->x48; return 0; }
    unsigned long long h = 0;
    HIPCHK(hipSetDevice(s->dev));
    HIPCHK(hipMemcpyAsync(&h, s->dX48, sizeof h, hipMemcpyDeviceToHost, s->stream));
    HIPCHK(hipStreamSynchronize(s->stream));
    *x = h;
    return 0;
}
