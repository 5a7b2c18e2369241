// Internal interface between the host engine (mdqt_engine.cpp) and the gfx950 kernels
// (mdqt_kernels.hip).  Plain structs passed BY VALUE as kernel arguments (no __constant__
// globals: several contexts with different parameters may live in one process).
#pragma once
#include <hip/hip_runtime.h>
#if defined(__HIP__)
#include <hip/hip_ext.h>
#endif
#include <stdint.h>

namespace mdqt {

constexpr int NS = 12;          // numStates, SpeedUp:153
constexpr int NBINS = 2001;     // SpeedUp:120-123
constexpr int MAXSUB = 32;      // substeps fused into one launch (ratio = 25 at density 2)
constexpr int NSTATIC = 20;     // static off-diagonal entries of M = I - i h H (App. A)
// Gaussian KDE of the velocity distributions (SpeedUp:958-979; the tagging programs' QTT:1072):
// exp(-V2 d^2), V2 = 1 / (2 0.002^2).  exp(x) is exactly +0 for x < -745.14 (below half the
// smallest subnormal), so a term with |d| >= kKdeSkip (V2 d^2 >= 746.9) adds an exact zero and the
// KDE kernels skip it; the assert ties the threshold to the bandwidth.
constexpr double kKdeV2 = 1. / (2. * 0.002 * 0.002);
constexpr double kKdeSkip = 0.0773;
static_assert(kKdeV2 * kKdeSkip * kKdeSkip * (1. - 1e-12) >= 746.0, "KDE skip threshold must lie beyond exp's underflow");

// Static couplings of the non-Hermitian Hamiltonian, as (row, col) of M; order of this
// table is the index used by the kernels (SpeedUp:1206-1215, cs[] at :1163-1180).
constexpr int kStaticRC[NSTATIC][2] = {
    {0, 3}, {0, 5}, {1, 2}, {1, 4}, {2, 1}, {2, 9}, {2, 11}, {3, 0}, {3, 8}, {3, 10},
    {4, 1}, {4, 7}, {5, 0}, {5, 6}, {6, 5}, {7, 4}, {8, 3}, {9, 2}, {10, 3}, {11, 2}};

// Constants of qstep() (SpeedUp:438-717), all precomputed on the host with the reference's
// own operation order so that device and oracle agree bit for bit where the math allows.
struct QTConst {
    double dtQ, gamToE;         // quantumTimestep, gamToEinsteinFreq (:79, :84)
    double h, dtHalf, invh;     // dtQ*gamToE, dtQ*gamToE/2, 1/(dtQ*gamToE)  (:525-567)
    double pv2q;                // plasVelToQuantVel (:85)
    double kRat, r;             // :146-147
    double det, detDP;          // detuning, detuningDP (:70-71)
    double kickS, kickD;        // 1*vKick*Om, vKickDP*(OmDP/r) (:503)
    double vKick, vKickDP;      // jump kicks (:589-610)
    double pD;                  // r/(r+1): D-decay branch probability (:589)
    double dP[4];               // decayMatrix diagonal on P levels 2..5 (:1203)
    double hdP[4];              // imag of hamDecayTerm diagonal on P levels (:1202)
    double hdPh[4];             // h dP[k]: qt_math 2 form of dp (= FastTab::hdp of the P levels)
    double a8, a11;             // OmDP/2*gs[8]/sqrt(r), OmDP/2*gs[11]/sqrt(r) (:508)
    double Mre[NSTATIC], Mim[NSTATIC];   // static off-diagonal M entries
    double thS3, thS4;          // gs[2]^2, gs[4]^2 (S-decay target thresholds)
    double thD[4][2];           // cumulative D-decay thresholds per P level (:612-697)
    double gs[18];
    double kickmax;             // bound on one substep's velocity kick (recoil or optical, model 0;
                                // |w|, |w_c| <= 4): the lane kernel's coupling-phase bound
    int renorm;                 // reNormalizewvFns (:706-712)
    int im01;                   // host: every static M entry of the lane table's slots 0 and 1 is
                                // purely imaginary (Re == +-0: -i h H with real couplings), so the
                                // FAST lane kernel drops their real-part FMAs (k_substeps_lanes_im)
    int model;                  // QT model (QTModel): level scheme, couplings and jump rule
    uint32_t seed, job;         // Philox key
};

// Per-lane tables of the lane-per-state QT kernel (16 lanes per ion, lane k <-> state k).
// Row k of M has its diagonal and up to three off-diagonal entries, in slots A < B < C by
// column; `order` says where the diagonal falls in the ascending-column sum:
//   0: D,A,B   1: A,D,B,C   2: A,D   3: A,B,D
struct LaneTab {
    int colA[16], colB[16], colC[16];
    int order[16], hasB[16], hasC[16];
    int dynB[16], dynC[16];      // slot holds a time-dependent entry: 1 = (8,5)/(9,4) form, 2 = (5,8)/(4,9)
    double cAre[16], cAim[16], cBre[16], cBim[16], cCre[16], cCim[16];   // static M entries
    double dynScale[16];         // a8 or a11 for the dynamic slot of rows 4, 5, 8, 9
    double gA[16], gB[16];       // optical-kick weights of rho_im(w_k, w_colA/colB) (:503)
    double dP[16];               // decayMatrix diagonal (0 off the P levels)
    double hd[16];               // imag of hamDecayTerm diagonal (0 off the P levels)
};

// qt_math 2 (reassociated QT arithmetic, mdqt_qtfast.hip): row k of M = I - i h H as its
// diagonal plus three off-diagonal slots with source states kFastCol[k][t] (unused slots point
// at k itself, or for model 0 at the zero state NS, with a zero coefficient; the time-dependent
// entry of rows 4, 5, 8, 9 sits in slot 2).  Both QT kernels evaluate every row as the same fixed
// FMA chain over these slots, so the thread-per-ion and lane-per-state forms stay bit-identical.
//
// Model 0's lane layout (lane-per-state kernel): the coupling graph (S-P and P-D edges, every P
// level of degree 3) is bipartite and splits into three matchings; states are placed on the 16
// lanes of an ion's row so that the matchings are lane ^ 2, lane + 8 (mod 16) and lane ^ 1 —
// three DPP moves (quad_perm, row_ror:8, quad_perm) instead of an LDS gather:
//   lane : 0  1  2  3  4  5  6  7  8  9  10 11 12 13 14 15
//   state: 2  1  9  4  3  0  8  5  11 -  -  7  10 -  -  6     (- : zero lanes; 9 = y, 10 = z)
// Slot 0 = lane ^ 2, slot 1 = lane + 8, slot 2 = lane ^ 1 (it carries the time-dependent
// couplings 4-9 and 5-8).  The sums over lanes (dp, kick, norm) follow lane order.
//
// QT models (mdqt_params.qt_model): 0 = the SpeedUp Sr+ 12-level laser cooling (default);
// the optical-pumping ("spin tagging") variants, one per reference program family:
//   1 = 408 nm linear, 7 levels   randomFrozenStartTag408Linear.cpp:396, MonteCarloFollowedByQTTagging408Linear.cpp:555
//   2 = 408 nm quad,   7 levels   randomFrozenStartTag408Quad.cpp (qstep :399: 2 couplings)
//   3 = 422 nm linear, 5 levels   randomFrozenStartTag422Linear.cpp:390, MonteCarloFollowedByQTTagging422Linear.cpp:552
// Levels of the pumping models: 0 S-1/2, 1 S+1/2, P levels from 2, then one D level (6 or 4).
// They have no optical-force kick, no time-dependent coupling and no jump kick; the kernels
// are the same template with another sparse H (FastTab) and jump table (jump_target_pump).
constexpr int NMODELS = 4;
constexpr int kModelStates[NMODELS] = {12, 7, 7, 5};
constexpr int kFastColM[NMODELS][NS][3] = {
    {{5, 12, 3}, {4, 12, 2}, {9, 11, 1}, {8, 10, 0}, {1, 7, 9}, {0, 6, 8},
     {12, 5, 12}, {12, 4, 12}, {3, 12, 5}, {2, 12, 4}, {12, 3, 12}, {12, 2, 12}},
    {{2, 4, 0}, {3, 5, 1}, {0, 2, 2}, {1, 3, 3}, {0, 4, 4}, {1, 5, 5},
     {6, 6, 6}, {7, 7, 7}, {8, 8, 8}, {9, 9, 9}, {10, 10, 10}, {11, 11, 11}},
    {{4, 0, 0}, {5, 1, 1}, {2, 2, 2}, {3, 3, 3}, {0, 4, 4}, {1, 5, 5},
     {6, 6, 6}, {7, 7, 7}, {8, 8, 8}, {9, 9, 9}, {10, 10, 10}, {11, 11, 11}},
    {{3, 0, 0}, {2, 1, 1}, {1, 2, 2}, {0, 3, 3}, {4, 4, 4}, {5, 5, 5},
     {6, 6, 6}, {7, 7, 7}, {8, 8, 8}, {9, 9, 9}, {10, 10, 10}, {11, 11, 11}}};
inline constexpr const int (&kFastCol)[NS][3] = kFastColM[0];
// model 0 lane layout (see above): state of lane l / lane of state k, as 4-bit fields (0xF: none)
constexpr uint64_t kStateOfLane0 = 0x6FFA7FFB58034912ull;   // lanes 15..0: 6 F F A 7 F F B 5 8 0 3 4 9 1 2
constexpr uint64_t kLaneOfState0 = 0x8C26BF734015ull;      // states 11..0: 8 C 2 6 B F 7 3 4 0 1 5
__host__ __device__ constexpr int state_of_lane0(int l) { return (int)((kStateOfLane0 >> (4 * l)) & 0xF); }
__host__ __device__ constexpr int lane_of_state0(int k) { return (int)((kLaneOfState0 >> (4 * k)) & 0xF); }
constexpr bool layout0_consistent() {      // slot j of state k's lane reads the lane of kFastColM[0][k][j]
    for (int k = 0; k < NS; ++k) {
        const int l = lane_of_state0(k);
        if (state_of_lane0(l) != k) return false;
        const int part[3] = {l ^ 2, (l + 8) & 15, l ^ 1};
        for (int j = 0; j < 3; ++j) {
            const int ps = state_of_lane0(part[j]);
            if ((ps >= NS ? NS : ps) != kFastColM[0][k][j]) return false;
        }
    }
    return true;
}
static_assert(layout0_consistent(), "model 0 lane layout and kFastColM[0] disagree");
struct FastTab {
    int col[3][16];              // kFastCol, lanes 12..15 point at themselves
    double cre[3][16], cim[3][16];   // static M entries of the slots (0 for unused / dynamic)
    double dms[16], dmc[16];     // slot 2 += {dms sin(phi), dmc cos(phi)} (rows 4, 5, 8, 9)
    double mre[16];              // Re M_kk = 1 + h Im(hamDecayTerm_kk)
    double mi0[16], mi1[16];     // Im M_kk = mi0 + mi1 u, u = velQuant + expDetuning (:506-510)
    double hdp[16];              // h decayMatrix_kk (P levels), 0 elsewhere: dp = sum hdp |y|^2
    double kw[3][16];            // optical-kick weight of Im(y_k conj(y_slot)), sign and scale folded (:503)
    double cphi;                 // 2 (1 + kRat) gamToE: phi = u cphi tPart (:508)
    double dt2;                  // (dtQ/2)^2 of step_R's first substep (:372-378)
};

struct SubstepArgs {
    double* R;          // this rank's slab of the gathered positions, [3][S]
    double* V;          // [3][S]
    double* F;          // [3][S]
    const double* Fpart;// if nseg > 1: force partials [nseg][3][S] summed here (in segment
    int nseg;           //   order) into F before the first substep, and F is written back
    double* psi;        // [24][S]: component-major (re0, im0, re1, ... im11)
    double* tPart;      // [S]
    int n;              // ions in this slab
    int S;              // slab stride (doubles)
    uint64_t gid0;      // global id of local ion 0
    uint64_t q0;        // qstep index of the first substep
    int nsub, do_step, do_qt;
    const double* U;    // rng_mode 0 (drand48 reference order): uniforms [5][S] of this substep
                        // (nsub == 1), from k_d48_resolve; nullptr = Philox stream
    int* oor;           // set to 1 if a final position leaves [-L/8, 9L/8] (see ForceArgs::oor)
    double L;
    double t[MAXSUB];       // global time at each substep (t before qstep advances it)
    double expDet[MAXSUB];  // expDetuning(t) (:447)
    uint32_t movmask;       // bit s: t[s] > 0 (step_R's moving branch, :360); set by the host
    int expdet_zero;        // every expDet[s] == 0 (fracOfSig = 0, the default)
    // overlapped / fused MD step (lane kernel, world 1): the force work runs concurrently (another
    // stream, or the first workgroups of k_md_step) and counts its finished tile pairs per tile in
    // arrive[ntiles]; this launch does its prologue, then waits until arrive[tile of its ions] >=
    // arrive_target before it reads the force partials (write-through stores there, L1-bypassing
    // loads here: mdqt_pairs.hpp n3_tile)
    const unsigned long long* arrive;
    unsigned long long arrive_target;
    int* spin_err;          // set if the wait gave up (bounded spin)
    int arrive_sleep;       // s_sleep 1 (64 cycles) units between polls (2)
    QTConst qc;
};

struct ForceArgs {
    const double* Rall; // gathered positions [world][3][S]
    double* Fpart;      // [nseg][3][S]: partial sums of the owned rows per j-segment
    int N, S;           // ions, slab stride
    int row_lo, nrows;  // owned global rows [row_lo, row_lo + nrows)
    int nseg, seglen;   // j segmentation (a function of N only)
    double L, lDeb, Rcut;
    double invlDeb;     // 1./lDeb (the reference recomputes it per pair; same IEEE value)
    double micT;        // smallest d with fl(d/L) >= 0.5: round(dx/L) = [dx >= micT] - [dx <= -micT]
    double micGuard;    // |dx| below this is inside the threshold rule's validity (|dx/L| < 1.5)
    int variant;        // 0 = exact (the reference's operations), 1 = fast (rsqrt/reciprocal form)
    int guard;          // positions may have left [-L/8, 9L/8] (set_state input or a device
                        // report): range-check every pair, far separations take the division form
};

// 1/sqrt(x): v_rsq_f64 (2^-24 relative on gfx950, tools/rsq_precision.hip) refined by one
// third-order step r (1 + e/2 + 3e^2/8), e = 1 - x r^2: 1.7e-16 max relative error measured
// (two Newton steps: 2.4e-16) in 5 dependent operations instead of 7
__device__ __forceinline__ double rsq3(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double q = __builtin_amdgcn_rsq(x);
#else
    const double q = 1. / sqrt(x);                 // host parse of device code only
#endif
    const double e = fma(-x, q * q, 1.0);
    return fma(q * e, fma(e, 0.375, 0.5), q);
}

// e^x for x = -r/lDeb in [-L/(2 lDeb), 0] (no overflow, no subnormal results for any box the
// reference runs): Cody-Waite x = n ln2 + r, |r| <= ln2/2, then the degree-11 minimax polynomial
// of e^r on [-ln2/2, ln2/2] (relative approximation error 3.1e-18; Remez exchange in 60-digit
// arithmetic, coefficients rounded to double) in FMA Horner form, exponent shift: <= 1.1 ulp vs
// the exact value over the range (two FMAs fewer per pair than a degree-13 Taylor polynomial).
__device__ __forceinline__ double exp_neg(double x) {
    const double n = __builtin_rint(x * 1.4426950408889634);
    double r = fma(-n, 0x1.62e42fefa39efp-1, x);
    r = fma(-n, 0x1.abc9e3b39803fp-56, r);
    double p = 2.4994304884817207e-08;
    p = fma(p, r, 2.7632293279459877e-07);
    p = fma(p, r, 2.7557622530872255e-06);
    p = fma(p, r, 2.4801486521427463e-05);
    p = fma(p, r, 0.00019841269432679237);
    p = fma(p, r, 0.0013888888951223987);
    p = fma(p, r, 0.00833333333355927);
    p = fma(p, r, 0.04166666666649277);
    p = fma(p, r, 0.1666666666666617);
    p = fma(p, r, 0.5000000000000018);
    p = fma(p, r, 1.0);
    p = fma(p, r, 1.0);
    return ldexp(p, (int)n);
}

// 2^t for t = -(r/lDeb) log2(e) <= 0 (the pair kernels' Yukawa factor e^(-r/lDeb) = 2^t, t formed
// as r * (-log2(e)/lDeb)): n = rint(t), f = t - n exactly (|f| <= 1/2, no reduction constant to
// round), then the degree-11 minimax-type polynomial of 2^f on [-1/2, 1/2] (Chebyshev fit in
// 50-digit arithmetic, coefficients rounded to double; <= 1.14 ulp with double FMA Horner),
// exponent shift.  Two operations fewer than exp_neg's Cody-Waite form; the only rounding before
// the polynomial is t's own, the same size as x = -r/lDeb's in exp_neg.
__device__ __forceinline__ double exp2_neg(double t) {
    const double n = __builtin_rint(t);
    const double f = t - n;
    double p = 0x1.e9ec1fcb69a7fp-32;
    p = fma(p, f, 0x1.e6228acd1c6e5p-28);
    p = fma(p, f, 0x1.b524ebd13a55fp-24);
    p = fma(p, f, 0x1.62bfc2c86d700p-20);
    p = fma(p, f, 0x1.ffcbfc6da6ed1p-17);
    p = fma(p, f, 0x1.430913112c61bp-13);
    p = fma(p, f, 0x1.5d87fe78a3f9cp-10);
    p = fma(p, f, 0x1.3b2ab6fb9f1a5p-7);
    p = fma(p, f, 0x1.c6b08d704a0c6p-5);
    p = fma(p, f, 0x1.ebfbdff82c5aep-3);
    p = fma(p, f, 0x1.62e42fefa39efp-1);
    p = fma(p, f, 1.0);
    return ldexp(p, (int)n);
}
constexpr double kNegLog2e = -1.4426950408889634;   // -log2(e)

// Far tile pairs of the Newton-3 blocks (box gap >= the far radius, mdqt_engine.cpp far_radius):
// every pair term there is below g(r_far), so a term error of relative size kFarRelErr is below
// g(r_far) kFarRelErr and an ion's force moves by at most (N - 1) g(r_far) kFarRelErr (<= 1e-13 by
// the choice of r_far).  Their pair form: rsq1 (v_rsq_f64 + ONE Newton step: 1e-14 relative) and
// 2^f by a degree-6 Chebyshev fit on [-1/2, 1/2] (2.6e-9 relative in double Horner, mpmath fit,
// measured on 4,001 points) — 6 operations fewer per pair than the exact form.
constexpr double kFarRelErr = 3e-9;
// The mid tier (round 4, sub-tile groups >= r_mid apart): rsq1 — relative error 1.5 e^2 + 2u for the
// raw rsq's e <= kRsqRawErr: <= kRsq1RelErr — and 2^t by the 64-entry table with a degree-4 series
// (2.53e-15 measured, + the table entry's and the product's rounding: kTab4RelErr).  t carries ri's
// error times r/lDeb, the force factor 3 ri's: a term is within (r/lDeb + 3)(kRsq1RelErr + 2^-52) +
// kTab4RelErr of itself (mdqt_engine.cpp far_err, level 5).
constexpr double kRsq1RelErr = 2.2e-14;
// 2^t of the exact (and mid) pair forms by the 64-entry LDS table (mdqt_pairs.hpp exp2_neg_cut_tab)
#ifndef MDQT_EXP_TAB
#define MDQT_EXP_TAB 1   // A/B round 4 (plan-based block kernel): C3 -3.5 %, C5 -0.8 %, N = 1M +0.3 %; round 3: C2 MD step -0.2 us
#endif
constexpr double kTab4RelErr = 4e-15;
__device__ __forceinline__ double rsq1(double x) {
#if defined(__HIP_DEVICE_COMPILE__)
    const double q = __builtin_amdgcn_rsq(x);
#else
    const double q = 1. / sqrt(x);
#endif
    const double e = fma(-x, q * q, 1.0);
    return fma(0.5 * q, e, q);
}
// The very-far tier (box gap >= r_vfar): the raw v_rsq_f64 (relative error <= kRsqRawErr: measured
// 2^-24 by tools/rsq_precision.hip over r^2 in [1e-4, 1e6], checked by a GPU test; twice that here)
// and a degree-5 fit of 2^f (1.02e-7 relative).  A term at distance r is then within
// ((r/lDeb + 3) kRsqRawErr + kExp5RelErr) of itself relatively — r/lDeb from t = r log2(e)/lDeb
// carrying ri's error into 2^t, 3 from ri^3 — and g(r) times that factor decreases in r, so
// (N - 1) g(r_vfar) ((r_vfar/lDeb + 3) kRsqRawErr + kExp5RelErr) bounds every ion (far_radius).
constexpr double kRsqRawErr = 0x1p-23;
constexpr double kExp5RelErr = 1.1e-7;
// The ultra-far tier (box gap >= r_ufar): the raw v_rsq_f64 and 2^t by v_exp_f32 on t rounded to
// float (relative 2^-24): a term is within (r/lDeb) (kRsqRawErr + 2^-24) + 3 kRsqRawErr +
// kExp2fRelErr of itself (kExp2fRelErr: twice what tools/exp2f_precision measures, re-checked by a
// GPU test).  f32's range holds 2^t down to t = -126: r <= 87 lDeb, beyond every L/2 it serves.
constexpr double kExp2fRelErr = 0x1p-22;
// The ultra-far tier in f32 (MDQT_UFAR32, round 3; round 5: relative to J's first ion, packed): a
// uniform-image tile pair's sub-tile group whose sub-boxes are >= r_ufar32 apart — and whose gap g is
// at least the J tile's raw box diagonal D (k_n3b_plan) — evaluates its pair terms in f32: the J tile
// staged as fl32(xj - c_J), c_J its first ion, the lane's ion as fl32(xi - n L - c_J), dx their f32
// difference; r^2 by f32 FMAs, v_rsq_f32 (<= kRsqF32RelErr = 1 ulp, measured by tools/rsq_precision
// and a GPU test), t = (r^2 ri) cf with cf = fl32(-log2(e)/lDeb), v_exp_f32, then the force factor and
// the three products in f32; the i side summed in two f32 partials of 8 steps, then in f64; the j side
// rotated along the wave over the 16 steps (one ds_add_f64 per component).  With u = 2^-24, per axis
// |ddx| <= u (|xi - n L - c_J| + |xj - c_J| + |dx|), and |xi - n L - c_J| <= r + D, |xj - c_J| <= D, so
// |ddx| <= u (2 r + 2 D) <= 4 u r as a vector (D <= g <= r).  To first order: r^2 8u + 3u = 11u,
// ri 5.5u + 2u = 7.5u, r 19.5u, t 21.5u — so 2^t is within (r/lDeb) 21.5u + kExp2fRelErr — the force
// factor ((ri + invl) 9.5u, times 2^t 1u, ri^2 16u, product 1u) 27.5u more, the product with dx 5u;
// each 16-term f32 sum adds 15u: a term is within (r/lDeb) 22u + 52u of itself (kUfar32A, kUfar32B,
// rounded up).  The cutoff is decided on the f32 r^2 (<= 11u off): pairs within 6u Rcut of L/2 may
// land on either side, each at most g(Rcut (1 - 2^-20)) — so far_radius_l's level 4 bounds every ion
// by (N - 1) g(r) err(r) + (N - 1) g(Rcut (1 - 2^-20)), and the tier is off where that cannot meet
// 10^-k (C5: N g(L/2) is ~1e-8; N = 1e6 at C2's parameters: ~5e-16).  force_form_mode 1 (round 6) has
// no such term: the plan gives a group the f32 form only if its far distance is below Rcut (1 - 2^-20)
// (N3BArgs::u32lim2), so its f32 r^2 never decides a cutoff.
#ifndef MDQT_UFAR32
#define MDQT_UFAR32 1
#endif
constexpr double kRsqF32RelErr = 0x1p-23;
constexpr double kUfar32A = 22. * 0x1p-24;
constexpr double kUfar32B = 52. * 0x1p-24;
// a term's relative error in the pair form of plan level e (0 exact, 1 mid, 2 far, 3 very far, 4 ultra
// far, 5 ultra far in f32) as kFormErrA[e] r/lDeb + kFormErrB[e] (mdqt_engine.cpp far_err; the measured
// form bound of k_n3b_plan, force_form_mode 1)
constexpr double kFormErrA[6] = {0., kRsq1RelErr + 0x1p-52, 0., kRsqRawErr, kRsqRawErr + 0x1p-24, kUfar32A};
constexpr double kFormErrB[6] = {0., 3. * (kRsq1RelErr + 0x1p-52) + kTab4RelErr, kFarRelErr,
                                 3. * kRsqRawErr + kExp5RelErr, 3. * kRsqRawErr + kExp2fRelErr, kUfar32B};
__device__ __forceinline__ double exp2_neg_cut5(double t, bool keep) {
    const double n = __builtin_rint(t);
    const double f = t - n;
    double p = 0x1.5f0890162a90ap-10;
    p = fma(p, f, 0x1.3d10705276a1dp-7);
    p = fma(p, f, 0x1.c6af6cdbbdcc7p-5);
    p = fma(p, f, 0x1.ebf906e26e833p-3);
    p = fma(p, f, 0x1.62e4302fc626ep-1);
    p = fma(p, f, 0x1.0000014413897p+0);
    return ldexp(p, keep ? (int)n : -1100);
}
__device__ __forceinline__ double exp2_neg_cut6(double t, bool keep) {
    const double n = __builtin_rint(t);
    const double f = t - n;
    double p = 0x1.443fffc90db59p-13;
    p = fma(p, f, 0x1.5f48c04f62e50p-10);
    p = fma(p, f, 0x1.3b2a1b7152befp-7);
    p = fma(p, f, 0x1.c6aecc669b6ddp-5);
    p = fma(p, f, 0x1.ebfbe045f4d3cp-3);
    p = fma(p, f, 0x1.62e430d034702p-1);
    p = fma(p, f, 1.0);
    return ldexp(p, keep ? (int)n : -1100);
}
// exp2_neg with a cutoff folded into the exponent shift: 0 (2^-1100 underflows) unless keep —
// one 32-bit select instead of a 64-bit one on the result.  For finite t only (the caller's
// r = 0 case must not occur: the Newton-3 tile kernels have no self pairs, distinct pad ions).
__device__ __forceinline__ double exp2_neg_cut(double t, bool keep) {
    const double n = __builtin_rint(t);
    const double f = t - n;
    double p = 0x1.e9ec1fcb69a7fp-32;
    p = fma(p, f, 0x1.e6228acd1c6e5p-28);
    p = fma(p, f, 0x1.b524ebd13a55fp-24);
    p = fma(p, f, 0x1.62bfc2c86d700p-20);
    p = fma(p, f, 0x1.ffcbfc6da6ed1p-17);
    p = fma(p, f, 0x1.430913112c61bp-13);
    p = fma(p, f, 0x1.5d87fe78a3f9cp-10);
    p = fma(p, f, 0x1.3b2ab6fb9f1a5p-7);
    p = fma(p, f, 0x1.c6b08d704a0c6p-5);
    p = fma(p, f, 0x1.ebfbdff82c5aep-3);
    p = fma(p, f, 0x1.62e42fefa39efp-1);
    p = fma(p, f, 1.0);
    return ldexp(p, keep ? (int)n : -1100);
}

// Canonical sum of nseg partials p[0], p[stride], ... : eight interleaved accumulators
// (partial s goes to s % 8, ascending) combined as ((a0+a1)+(a2+a3))+((a4+a5)+(a6+a7)).  One
// fixed order wherever it is evaluated (deterministic); independent loads, short chains.
__device__ __forceinline__ double seg_sum(const double* __restrict__ p, size_t stride, int nseg) {
    double a[8] = {0., 0., 0., 0., 0., 0., 0., 0.};
    int s = 0;
    for (; s + 8 <= nseg; s += 8) {
#pragma unroll
        for (int q = 0; q < 8; ++q) a[q] += p[(size_t)(s + q) * stride];
    }
#pragma unroll
    for (int q = 0; q < 8; ++q)
        if (s + q < nseg) a[q] += p[(size_t)(s + q) * stride];
    return ((a[0] + a[1]) + (a[2] + a[3])) + ((a[4] + a[5]) + (a[6] + a[7]));
}

// THE canonical sum of the nseg force partials of one ion component (MDQT engine): sixteen
// strided partial sums, q_k = (((0 + p[k]) + p[k + 16]) + p[k + 32]) + ... (k = 0..15, the
// slots < nseg), combined by the lane kernel's DPP tree
//   (((q0 + q1) + (q2 + q3)) + ((q4 + q5) + (q6 + q7))) + (((q8 + q9) + ...) + ((q12 + q13) + (q14 + q15))).
// The lane-per-state QT kernel evaluates it distributed over an ion's 16 lanes (lane k: q_k, all
// of its loads in flight at once), the thread-per-ion kernels and k_reduce_segments serially:
// the same operations, so every consumer of the partials sees the same F bit for bit.
__device__ __forceinline__ double slot_sum16_partial(const double* __restrict__ p, size_t stride, int nseg, int k) {
    double q = 0.;
    for (int s = k; s < nseg; s += 16) q = q + p[(size_t)s * stride];
    return q;
}
__device__ __forceinline__ double tree16_sum(const double* q) {
    return (((q[0] + q[1]) + (q[2] + q[3])) + ((q[4] + q[5]) + (q[6] + q[7]))) +
           (((q[8] + q[9]) + (q[10] + q[11])) + ((q[12] + q[13]) + (q[14] + q[15])));
}
__device__ __forceinline__ double slot_sum16(const double* __restrict__ p, size_t stride, int nseg) {
    double q[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) q[k] = slot_sum16_partial(p, stride, nseg, k);
    return tree16_sum(q);
}

// Newton-3 tile-pair scheme (world_size 1): one workgroup of 4 waves per 64x64 tile pair
// (I <= J); partials go to slot J (rows of I) and slot I (rows of J), the diagonal tile's two
// sides to slot I.  F = canonical sum of the ntiles slots (seg_sum), like the row segments.
struct N3Args {
    const double* R;    // [3][S] (world_size 1)
    double* P;          // [ntiles][3][S]
    const int2* pairs;  // (I, J) of every workgroup; I's bits 28-31: a part of the tile pair's rotation
                        // steps (mdqt_pairs.hpp n3_tile; later parts write the extra slots from ntiles on)
    int N, S, ntiles, npairs;
    double L, lDeb, Rcut, invlDeb, micT, micGuard;
    int guard;          // as ForceArgs::guard (exact variant only; the fast one needs no guard)
    double rc2;         // variant 2: smallest double x with sqrt(x) >= Rcut (pair kept iff r2 < rc2)
    unsigned long long* arrive;   // [ntiles] arrival counts (overlapped / fused MD step): a finished
                                  // tile pair (I, J) adds 1 to arrive[I] and arrive[J] after its
                                  // write-through slot stores — T per tile per launch; nullptr = off
};

// Newton-3 over block pairs (mdqt_forces.hip k_pairs_n3b): blocks of 16 tiles, cyclic half
// shell of block distances, slots [nd + R][3][Npad] (j-slots by distance, i-slots by run).
// A rank runs the workgroups of blocks [Plo, Phi); k_n3b_reduce sums the slots it wrote.
struct N3BArgs {
    const double* Rall; // gathered positions [world][3][S]
    double* slots;      // [nd + R][3][Npad]
    int N, S, T, Npad;  // ions, slab stride, tiles, T * 64
    int NB, nd, R, runlen;   // blocks, half-shell distances NB/2 + 1, runs per block, distances per run
    int Plo, Phi;       // this rank's blocks
    double L, lDeb, Rcut, invlDeb, micT, micGuard;
    int guard;
    // spatial order (mdqt_sort.hip): tiles are 64 consecutive ions of the Hilbert order
    int use_sort;       // 1: positions from Rs, slots by sorted index, tile pairs beyond L/2 skipped;
                        // 2: the same order, nothing skipped (tests: bit-identical to 1)
    int pairs;          // 1: the paired-wave block kernel (k_pairs_n3b_pw; option "force_n3b_pairs"), 0: k_pairs_n3b
    int ax1;            // 1: the one-axis per-pair image instance where the skip radius reaches the image
                        // boundary (launch_forces_n3b; option "force_ax1"), 0: every per-pair image on all axes
    const double* Rs;   // [3][Npad] positions in sorted order
    const int* perm;    // sorted index -> ion
    const double* boxes;// [12][T]: tile center (x, y, z), half extents, raw coordinate min, max
    double Rmid;        // sub-tile groups >= Rmid apart take the mid pair form (rsq1 + table 2^t, ~2e-14
                        // relative; forces only, MDQT_EXP_TAB); >= Rcut: never
    double Rfar;        // tile pairs whose boxes are >= Rfar apart take the far pair form (kFarRelErr;
                        // forces only, use_sort 1 or 2); >= Rcut: never
    double Rvfar;       // >= Rvfar apart: the very-far form (raw rsq, degree-5 2^f); >= Rcut: never
    double Rufar;       // >= Rufar apart: the ultra-far form (raw rsq, v_exp_f32); >= Rcut: never
    double Rufar32;     // >= Rufar32 apart (uniform image): the ultra-far form in f32 (MDQT_UFAR32)
    double rc2;         // Rcut^2: the very-far and ultra-far forms keep a pair iff r^2 < rc2 (r^2 in f64,
                        // as exact as the exact form's r < Rcut), not on their low-precision r
    double Rskip;       // force tile pairs whose boxes are >= Rskip apart are skipped (use_sort 1):
                        // Rcut exactly (every skipped pair is beyond L/2), or the error-bounded tail
                        // radius r_t < L/2 of mdqt_engine.cpp tail_radius (potentials: always Rcut)
    double* tailb;      // force_tail_mode 1: per 16-ion sub-tile [4T], the sum over the pairs the call
                        // drops inside L/2 (tail-skipped tile pairs, skipped sub-tile groups) of
                        // n_b g(sub-block gap) — the measured bound on what each of its ions loses
                        // (zeroed before the launch, summed by k_n3b_plan; nullptr: not measured)
    int formm;          // force_form_mode 1 (round 6): tailb also sums, over the sub-blocks evaluated in an
                        // error-bounded form, n_b g(gap) err_form(gap) — the forms' measured bound, enforced
                        // with the tail's (k_tail_max, k_tail_fix); the tier radii come from a density model
    double u32lim2;     // formm: (Rcut (1 - 2^-20))^2 — a group takes the f32 ultra-far form only if every
                        // pair of it is closer (its boxes' far distance in the minimum image, sub_far2), so
                        // the f32 r^2 never decides the cutoff (no a-priori cutoff term)
    const double* subboxes;   // [6][4T]: the 16-ion sub-tiles' centers and half extents (use_sort)
    uint2* plan;        // force calls in spatial order: [(Phi - Plo) nd][256] tile-pair words, then
                        // [(Phi - Plo) nd] J-step masks (.x), written by k_n3b_plan (launch_forces_n3b)
                        // and read by k_pairs_n3b; nullptr: classified in the block kernel (every
                        // sub-tile group exact; no tail sums)
    unsigned long long* tmask;   // with a plan: [T][tmw] bit db of J tile's words = the block kernel wrote J's
    int tmw;                     // j-slot db (a J step with work); k_n3b_reduce reads only those (nullptr: all)
};
struct SortArgs {
    const double* Rall; // gathered positions [world][3][S]
    int N, S, Npad;
    double L;
    uint32_t *keys, *keys2;  // [N] Hilbert keys, sorted keys
    int *ion, *perm;         // [N] identity, sorted index -> ion
    void* tmp;               // hipCUB radix-sort scratch
    size_t tmp_bytes;
    double* Rs;              // out [3][Npad]
    double* boxes;           // out [12][T]
    double* subboxes;        // out [6][4T]: the 16-ion sub-tiles' centers and half extents (or null)
};
hipError_t launch_spatial_order(const SortArgs& a, hipStream_t s);
size_t spatial_order_tmp_bytes(int N);
// ev0/ev1: the block kernel's own dispatch timestamps (timing on; k_pairs_n3b alone, not the plan or
// the reduction); marks (optional, the force-call breakdown): 3 events recorded after the plan, after the
// block kernel and after the slot reduction
hipError_t launch_forces_n3b(const N3BArgs& a, int variant, double* out, hipStream_t s, hipEvent_t ev0 = nullptr,
                             hipEvent_t ev1 = nullptr, hipEvent_t* marks = nullptr);
// force_tail_mode 1 (mdqt_forces.hip): the per-sub-tile tail sums [4T] against eps — st[0] running
// max of the tiles within eps, st[1] of all, st[2] tiles over eps (cumulative), st[3] this call's
// list length, st[4] measured calls — and the exact recomputation of the listed tiles' forces,
// written into `out` ([world][3][S], by ion) on the rank that owns the tile (0 on the others); pot: their
// potential rows U_i (component 0) instead
hipError_t launch_tail_max(const double* tailb, int T, double eps, unsigned long long* st, int* list, hipStream_t s);
hipError_t launch_tail_fix(const N3BArgs& a, const unsigned long long* st, const int* list, double* out,
                           hipStream_t s, bool pot = false);
// census of k_pairs_n3b's work by tile-pair class (mdqt_forces.hip k_n3b_census): out[2 kCensus]
constexpr int kCensus = 15;                 // (round 6: + 14 ufar_image)
// tiles per block of the Newton-3 block kernel (= its waves per workgroup): 8 (round 4, A/B vs 16:
// C3 -2.7 %, C5 -2.5 %, N = 1M -4.3 % per force call — three 8-wave workgroups per CU at 80 VGPRs
// instead of two 16-wave ones at 64: shorter J-step barriers, fewer spills; 4: slower)
#ifndef MDQT_N3B_BW
#define MDQT_N3B_BW 8
#endif
constexpr int kN3BBlock = MDQT_N3B_BW;
hipError_t launch_n3b_census(const N3BArgs& a, unsigned long long* out, hipStream_t s, unsigned long long* bw = nullptr,
                             unsigned long long* bal = nullptr);
hipError_t launch_sum_rank_chunks(const double* const* parts, int world, int rank, int S, double* F, hipStream_t s);

// ---- Monte-Carlo + MD analytics program (mdmc_kernels.hip) ----
struct MCArgs {
    double* R;          // [3][S]
    double* U;          // [N] per-particle potential energies (MCMD:123)
    double* D;          // [N] scratch: the candidate U'
    uint32_t* mt;       // [625]: std::mt19937 state words + position (in/out)
    unsigned long long* accepted;   // in/out
    int N, S, nsteps;
    double L, kappa, rCut, maxRStep, Gamma;
    double micT;        // smallest d with fl(d / L) >= 0.5: round(d/L) without a division, |d| < 1.25 L
    int fast;           // 1: reciprocal pair energy values (rsq, exp_neg; <= 2 ulp per pair), 0: the reference's ops;
                        //    both keep the reference's pair set: exact image, cutoff as r2 < rc2
    double rc2;         // smallest double x with sqrt(x) >= rCut
};
struct VVArgs {
    double* V;
    double* A;          // in: a(t) ; out: a(t + dt) = the canonical sum of the force slots
    const double* slots;   // [nslots][3][S] Newton-3 tile partials of a(t + dt)
    int nslots;
    const double* R;    // r(t + dt)
    double* Rn;         // out: r(t + 2 dt) = stepPositions of the next MDStep (pre-advanced)
    double L;
    const double* hits;        // [nhits][4] = (i, vx, vy, vz): this step's collisions (host-drawn)
    int nhits;
    int N, S, laser, oneAxis;
    double dt, p6, beta, sqrtn; // p6 = pow(10, -6), sqrtn = sqrt(n) (MCMD:491-496)
};
hipError_t launch_particle_potentials(const double* R, int N, int S, double L, double kappa, double rCut, double* U,
                                      hipStream_t s);
hipError_t launch_monte_carlo(const MCArgs& a, hipStream_t s);
hipError_t launch_vv_positions(const double* R, const double* V, const double* A, double* Rn, int N, int S, double dt,
                               double L, hipStream_t s);
hipError_t launch_vv_velocities(const VVArgs& a, hipStream_t s);   // + the collision scatter when nhits > 0
hipError_t launch_pair_hist(const double* R, int N, int S, double L, double step, int nbins, unsigned* hist,
                            hipStream_t s);
int autocorr_blocks(int N);
hipError_t launch_autocorr(const double* vs, int N, int T, double c2, double c4, double* part, double* out,
                           hipStream_t s);
hipError_t launch_temperatures(const double* V, int N, int S, double* out, hipStream_t s);
hipError_t launch_tag_moments(const double* V, const int* tags, int N, double* out, hipStream_t s);
hipError_t launch_anisotropize(double* V, int N, int S, double tpd, hipStream_t s);
hipError_t launch_store_velocities(const double* V, int N, int S, int T, int t, double* vs, hipStream_t s);
// error message of the C ABI (mdqt_last_error), shared by the mdmc_* entry points
int set_error(const char* fmt, ...);
// pumping-model QT tables for another engine (mdqt_engine.cpp; used by the MC + MD tagging programs)
void build_pump_program(int model, double detuning, double Om, double dtQ, double gamToE, double pv2q,
                        double decayRatio, uint32_t seed, uint32_t job, QTConst& q, FastTab& f);
// recordTaggedParticleMoments' velocity distribution of the tagged ions (QT tagging programs):
// out[c][j] = sum over tagged i (ascending) of exp(-V2 (vel_j - V[c][i])^2), vel_j = (j - 2000) 0.0025
constexpr int TKDE_BINS = 4001;
// bins vel_j = (j + bin0) 0.0025: bin0 = -2000 (the programs' init(), e.g. randomFrozenStartTag408Linear.cpp:306),
// 0 after their readConditions (:723 sets vel[i] = i 0.0025)
hipError_t launch_tagged_kde(const double* V, const int* tags, int N, int S, double* part, double* out, hipStream_t s,
                             int bin0 = -2000);
// one half of the pumping programs' leapfrog MD step (randomFrozenStartTag408Linear.cpp step(), :317-394):
// if kick != 0, V += kick F first (step_V); then step_R: R += DT V (moving) or R += DT V + DT2 F
// (t == 0), and the reinsertion into [0, L]
hipError_t launch_leapfrog_half(double* R, double* V, const double* F, int n, int S, double L, double DT, double DT2,
                                int moving, double kick, hipStream_t s);

// drand48 in the reference's order (SpeedUp:486, :575-687: ions in index order, 1 draw per
// ion, 4-5 for a quantum jump): one workgroup assigns every ion its uniforms from the single
// stream, by LCG jump-ahead from the stream state, restarting after each (rare) jump.
struct D48Args {
    const double* psi;         // [24][S]
    int n, S;
    unsigned long long* state; // device: drand48 X before this substep's first draw; advanced
    const unsigned long long* jA;   // [48] multiplier of 2^b steps
    const unsigned long long* jC;   // [48] increment of 2^b steps
    double* U;                 // out: [5][S]
    int fast;                  // qt_math of the substep kernel (0, 1, 2: dp must be bit-identical)
    QTConst qc;
};
hipError_t launch_d48_resolve(const D48Args& a, hipStream_t s);

// ---- launchers (mdqt_kernels.hip) ----
hipError_t launch_forces(const ForceArgs& a, hipStream_t s);
hipError_t launch_forces_n3(const N3Args& a, int variant, hipStream_t s, hipEvent_t ev0 = nullptr,
                            hipEvent_t ev1 = nullptr);
// Epotential on the Newton-3 tiles (world 1): pair potentials into slot p of a.P, plane stride S
// ([ntiles][S]: one component, a third of the force slots' memory)
hipError_t launch_potential_n3(const N3Args& a, int variant, hipStream_t s);
// Epotential on the Newton-3 blocks (world 1): per-ion row sums of u into out[S]; with a.plan on the force
// call's plan (skips, sub-tile groups, error-bounded forms; tail sums into a.tailb), else exact to L/2;
// ev0/ev1 (optional) time the block kernel
hipError_t launch_potential_n3b(const N3BArgs& a, int variant, double* out, hipStream_t s, hipEvent_t ev0 = nullptr,
                                hipEvent_t ev1 = nullptr);
// partial p of component c at Fpart + p * plane + c * S (plane 0: 3 S, the force layout)
hipError_t launch_reduce_segments(const double* Fpart, double* F, int nseg, int nrows, int S, int ncomp,
                                  hipStream_t s, size_t plane = 0);
hipError_t launch_potential_rows(const ForceArgs& a, hipStream_t s);   // Fpart[seg][0][i]
// mode: 0 = auto (lane-per-state below kLaneKernelMaxIons ions, thread-per-ion above),
//       1 = thread-per-ion, 2 = lane-per-state.  Both are bit-identical.
constexpr int kLaneKernelMaxIons = 98304;
// fast: qt_math 1 (FMA contraction, refined rsq) instead of the reference's exact operations
#if defined(__HIP__)
// Launch with the kernel's own dispatch timestamps written to (ev0, ev1) when timing is on
// (hipExtLaunchKernelGGL): the measured interval is the kernel itself, without the event
// packets' queue time that a pair of hipEventRecord calls around the launch adds.
template <typename... Args, typename F = void (*)(Args...)>
inline void launch_timed(F kernel, dim3 grid, dim3 block, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1,
                         Args... args) {
    if (ev0) hipExtLaunchKernelGGL(kernel, grid, block, 0, s, ev0, ev1, 0, args...);
    else hipLaunchKernelGGL(kernel, grid, block, 0, s, args...);
}
#endif

// The substep kernel instance a launch ran (mdqt_get_const "qt_kernel"; the launchers report it
// through `instance`): tests check which instance a configuration's production launch takes.
enum QTKernel : int {
    QTK_NONE = 0,
    QTK_LANES_IM_EDZ = 1,      // k_substeps_lanes_im<true, true, true>: model 0 FAST + IM01 + EDZ, no
                               // renormalisation (the C2 production launch)
    QTK_LANES_IM = 2,          // k_substeps_lanes_im<true, false>
    QTK_LANES_R_FAST = 3,      // k_substeps_lanes_r<true, true>
    QTK_LANES_R = 4,           // k_substeps_lanes_r<true, false>
    QTK_LANES_R_PUMP_FAST = 5, // k_substeps_lanes_r<false, true>
    QTK_LANES_R_PUMP = 6,      // k_substeps_lanes_r<false, false>
    QTK_LANES_IM_EDZ_RN = 7,   // k_substeps_lanes_im<true, true, false>: the same with reNormalizewvFns on
    QTK_THREAD_R = 10,         // k_substeps_r<model>: 10 + model
    QTK_MD_STEP = 20,          // k_md_step (one launch per MD step)
    QTK_EXACT_LANES = 30,      // k_substeps_lanes<fast>: 30 + qt_math
    QTK_EXACT_THREAD = 40,     // k_substeps<fast>: 40 + qt_math
};
// ev0/ev1 (optional): the kernel's own start/stop timestamps (hipExtLaunchKernelGGL)
hipError_t launch_substeps(const SubstepArgs& a, const LaneTab* tab, int mode, int fast, hipStream_t s,
                           hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr, int* instance = nullptr);
// qt_math 2: the reassociated kernels of mdqt_qtfast.hip (same modes as launch_substeps)
hipError_t launch_substeps_r(const SubstepArgs& a, const FastTab* tab, int mode, hipStream_t s,
                             hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr,
                             int* instance = nullptr);   // tab[0] by state, tab[1] by lane
// one MD step in one launch: Newton-3 tile pairs + the FAST lane QT kernel (mdqt_qtfast.hip
// k_md_step); f.arrive / a.arrive = the per-tile arrival counters, a.arrive_target their value
// after this launch's tile pairs
hipError_t launch_md_step(const N3Args& f, const SubstepArgs& a, const FastTab* tab, int variant, hipStream_t s,
                          hipEvent_t ev0 = nullptr, hipEvent_t ev1 = nullptr);
// measureSpinUps (randomFrozenStartTag408Linear.cpp:600, :422Linear) / tagParticles
// (MonteCarloFollowedByQTTagging408Linear.cpp:1022): tag[i] = 1 with probability of spin up
hipError_t launch_tag_spin_up(const double* psi, int n, int S, uint64_t gid0, uint64_t q, const QTConst& qc,
                              int* tags, hipStream_t s);
// deterministic sums: out[0] = sum vx; needs scratch >= 1024 doubles
// avg (optional, world 1): also avg[0] = sum / N on the device
hipError_t launch_sum_vx(const double* V, int n, double* out, hipStream_t s, double* avg = nullptr, int N = 0);
hipError_t launch_output_pack(const double* V, const double* psi, int n, int S, int model, double* out,
                              hipStream_t s);
// out[0..2] = sum 0.5 (vx-avg)^2, 0.5 vy^2, 0.5 vz^2 ; out[3] = sum of rows[0..nrows) of
// the potential partials reduced over segments (caller passes the reduced row buffer)
hipError_t launch_energy_sums(const double* V, int n, int S, const double* vxAvg,
                              const double* urow, double* out, hipStream_t s);
// KDE partials: P[ichunk][3][2001]; then reduce into Pout[3][2001] (unnormalised)
hipError_t launch_kde(const double* V, int n, int S, const double* vxAvg, double* Ppart,
                      int nchunk, double* Pout, hipStream_t s);

}  // namespace mdqt
