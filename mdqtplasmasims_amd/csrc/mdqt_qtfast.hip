// qt_math 2: the fused step()+qstep() substeps (SpeedUp:356-430, :438-717) with reassociated
// arithmetic, for throughput.  Same algorithm as mdqt_kernels.hip's k_substeps/_lanes, but
// every quantity is evaluated in the form that needs the fewest dependent instructions:
//
//   * row k of M = I - i h H is ONE fixed FMA chain: diagonal, then three off-diagonal slots
//     (FastTab; zero coefficients where a row has fewer entries), instead of the dense
//     product's ascending-column order;
//   * the RK stages work on d = s - y with s = M y / sqrt(1 - dp(y)) (k = d / h): y1 = w + d1/2,
//     y2 = w + d2/2, y3 = w + d3, w' = w + (d1 + 3 d2 + 3 d3 + d4)/8 — the reference's
//     k1 + 3k2 + 3k3 + k4 propagator (:525-567) without the 1/h and h factors;
//   * dp, the optical kick and the renormalisation norm are fixed-shape trees (the lane
//     kernel's DPP tree order), constants folded on the host (kick scale, h dP, 2(1+kRat)gamToE);
//   * step(): one coordinate per lane (lanes 0..11 and 14..15 x, 12 y, 13 z), exact operations.
//
// Results differ from the exact mode (qt_math 0) by rounding only (~1e-15 relative per
// substep; tests/test_gpu_parity.py bounds it against the oracle).  The thread-per-ion and
// lane-per-state kernels below perform the same operations in the same order: bit-identical.
#include "mdqt_device.hpp"
#include "mdqt_pairs.hpp"

#include <math.h>

#include <type_traits>

namespace mdqt {

// threads per workgroup of the lane-per-state kernels (16 lanes per ion)
#ifndef MDQT_LANE_WG
#define MDQT_LANE_WG 256
#endif
constexpr int kLaneWG = MDQT_LANE_WG;
static_assert(kLaneWG % 64 == 0 && kLaneWG <= 256, "lane kernel workgroup: whole waves, <= 256 threads");
static_assert(!MDQT_QT_SCTAB || kLaneWG >= 128, "the sincos table is staged by the first 128 threads");
// ions per wave of the lane kernels (diagnostic A/B builds only: MDQT_EXPT_ROWS 1 or 2 leave rows
// of 16 lanes idle — they shadow another row's ion without storing — so that a launch has 4 / 2x
// the waves at the same instructions per wave; the product keeps 4)
#ifndef MDQT_EXPT_ROWS
#define MDQT_EXPT_ROWS 4
#endif
constexpr int kRows = MDQT_EXPT_ROWS;
static_assert(kRows == 1 || kRows == 2 || kRows == 4, "ions per wave");
constexpr int kLaneIons = kLaneWG / 64 * kRows;      // ions per workgroup

__device__ __forceinline__ double rsq_nr(double x) { return rsq3(x); }   // 1/sqrt(x), mdqt_internal.hpp
__device__ __forceinline__ double nrm2(cxd y) { return fma(y.re, y.re, y.im * y.im); }
__device__ __forceinline__ double rho_im_r(cxd a, cxd b) { return fma(a.im, b.re, -(a.re * b.im)); }

// M_kk y + c0 y0 + c1 y1 + c2 y2, one chain per component
__device__ __forceinline__ cxd row_r(cxd md, cxd y, cxd c0, cxd y0, cxd c1, cxd y1, cxd c2, cxd y2) {
    double re = md.re * y.re, im = md.re * y.im;
    re = fma(-md.im, y.im, re);  im = fma(md.im, y.re, im);
    re = fma(c0.re, y0.re, re);  im = fma(c0.re, y0.im, im);
    re = fma(-c0.im, y0.im, re); im = fma(c0.im, y0.re, im);
    re = fma(c1.re, y1.re, re);  im = fma(c1.re, y1.im, im);
    re = fma(-c1.im, y1.im, re); im = fma(c1.im, y1.re, im);
    re = fma(c2.re, y2.re, re);  im = fma(c2.re, y2.im, im);
    re = fma(-c2.im, y2.im, re); im = fma(c2.im, y2.re, im);
    return {re, im};
}

// row_r when the static slots 0 and 1 are purely imaginary (c.re = +-0): their real-part FMAs
// add +-0 * y and are dropped — the same values up to the sign of an exact-zero result
__device__ __forceinline__ cxd row_r_im01(cxd md, cxd y, double c0im, cxd y0, double c1im, cxd y1, cxd c2, cxd y2) {
    double re = md.re * y.re, im = md.re * y.im;
    re = fma(-md.im, y.im, re);  im = fma(md.im, y.re, im);
    re = fma(-c0im, y0.im, re);  im = fma(c0im, y0.re, im);
    re = fma(-c1im, y1.im, re);  im = fma(c1im, y1.re, im);
    re = fma(c2.re, y2.re, re);  im = fma(c2.re, y2.im, im);
    re = fma(-c2.im, y2.im, re); im = fma(c2.im, y2.re, im);
    return {re, im};
}

__device__ __forceinline__ double kick_term(cxd w, cxd w0, cxd w1, cxd w2, double k0, double k1, double k2) {
    return fma(rho_im_r(w, w0), k0, fma(rho_im_r(w, w1), k1, rho_im_r(w, w2) * k2));
}

// sum of 16 values in the lane kernel's DPP tree order (row_shl 1, 2, 4, 8)
__device__ __forceinline__ double tree16(const double* v) {
    return (((v[0] + v[1]) + (v[2] + v[3])) + ((v[4] + v[5]) + (v[6] + v[7]))) +
           (((v[8] + v[9]) + (v[10] + v[11])) + ((v[12] + v[13]) + (v[14] + v[15])));
}
__device__ __forceinline__ double lane_tree16(double v) {
    double a = v + dpp<SHL(1)>(v);
    a = a + dpp<SHL(2)>(a);
    a = a + dpp<SHL(4)>(a);
    a = a + dpp<SHL(8)>(a);
    return dpp<BCAST(0)>(a);
}
#ifndef MDQT_NORM_Q
#define MDQT_NORM_Q 1
#endif
// renormalisation sum of the ion's 16 lanes: quads Q_m = (v_4m + v_4m+1) + (v_4m+2 + v_4m+3),
// then ((Q0 + Q1) + Q2) + Q3 (MDQT_NORM_Q; else the full DPP tree lane_tree16)
__device__ __forceinline__ double tree16n(const double* v) {
    if (!MDQT_NORM_Q) return tree16(v);
    double q[4];
#pragma unroll
    for (int m = 0; m < 4; ++m) q[m] = (v[4 * m] + v[4 * m + 1]) + (v[4 * m + 2] + v[4 * m + 3]);
    return ((q[0] + q[1]) + q[2]) + q[3];
}
// (T2 + T3) + (T4 + T5) of the ion's lanes 2..5, in every lane of the row
__device__ __forceinline__ double lane_sum_p(double T) {
    double a = T + dpp<SHL(1)>(T);
    a = a + dpp<SHL(2)>(a);
    return dpp<BCAST(2)>(a);
}

// step_R(dt/2) of one coordinate (:356-389), the reference's operations (step() stays bit-exact
// in every qt_math mode); `moving` = t > 0 (:360)
__device__ __forceinline__ double half_drift(double p, double v, double f, bool moving, double DT,
                                             double DT2, double L) {
    p = moving ? p + DT * v : p + (DT * v + DT2 * f);
    // (measured: one fma p + m L with m = +1 / -1 / 0 instead of the two conditional adds issues 6
    // instructions fewer per substep but lengthens the dependent chain — QT launch 21.3 -> 21.8 us,
    // A/B round 3; the reference's two adds are kept)
    if (p < 0) p += L;
    if (p > L) p -= L;
    return p;
}

// the quantum jump (:573-703), the exact-mode operations of mdqt_kernels.hip
__device__ __forceinline__ int jump_target(const QTConst& qc, double n3, double n4, double n5, double n6,
                                           double rand2, double randDOrS, double randDir, double rand3,
                                           double& kick) {
    const double tot = n3 + n4 + n5 + n6;
    const double prob3 = n3 / tot, prob4 = n4 / tot, prob5 = n5 / tot;
    const bool sDecay = !(randDOrS < qc.pD);
    if (!sDecay) kick = (randDir < 0.5) ? qc.vKickDP : -qc.vKickDP;
    else kick = (randDir < 0.5) ? qc.vKick : -qc.vKick;
    if (rand2 < prob3) {
        if (sDecay) return 1;
        return (rand3 < qc.thD[0][0]) ? 11 : (rand3 < qc.thD[0][1]) ? 10 : 9;
    } else if (rand2 < prob3 + prob4) {
        if (sDecay) return (rand3 < qc.thS3) ? 0 : 1;
        return (rand3 < qc.thD[1][0]) ? 10 : (rand3 < qc.thD[1][1]) ? 9 : 8;
    } else if (rand2 < prob3 + prob4 + prob5) {
        if (sDecay) return (rand3 < qc.thS4) ? 1 : 0;
        return (rand3 < qc.thD[2][0]) ? 9 : (rand3 < qc.thD[2][1]) ? 8 : 7;
    }
    if (sDecay) return 0;
    return (rand3 < qc.thD[3][0]) ? 8 : (rand3 < qc.thD[3][1]) ? 7 : 6;
}

// quantum jump of the optical-pumping models (no kick).  Draws in the reference's order: u1,
// rand2, randDOrS, then 408: randDir (unused), [rand3]; 422: [rand3] — i.e. rand3 is draw 4 for
// 408 (randomFrozenStartTag408Linear.cpp:521-590) and draw 3 for 422 (...422Linear.cpp:174-231)
__device__ __forceinline__ int jump_target_pump(const QTConst& qc, double n3, double n4, double n5, double n6,
                                                double rand2, double randDOrS, double d3, double d4,
                                                double& kick) {
    kick = 0.;
    const bool sDecay = !(randDOrS < qc.pD);
    if (qc.model == 3) {                            // 422: P levels 2, 3; D level 4
        const double tot = n3 + n4;
        const double prob3 = n3 / tot;
        if (rand2 < prob3) return sDecay ? ((d3 < 2. / 3) ? 1 : 0) : 4;
        return sDecay ? ((d3 < 2. / 3) ? 0 : 1) : 4;
    }
    const double tot = n3 + n4 + n5 + n6;           // 408: P levels 2..5; D level 6
    const double prob3 = n3 / tot, prob4 = n4 / tot, prob5 = n5 / tot;
    if (rand2 < prob3) return sDecay ? 0 : 6;
    if (rand2 < prob3 + prob4) return sDecay ? ((d4 < 2. / 3) ? 0 : 1) : 6;
    if (rand2 < prob3 + prob4 + prob5) return sDecay ? ((d4 < 1. / 3) ? 0 : 1) : 6;
    return sDecay ? 1 : 6;
}

__device__ __forceinline__ double sq(cxd y) { return y.re * y.re + y.im * y.im; }

// ------------------------------------------------------------------------------------------
// thread per ion
// ------------------------------------------------------------------------------------------
// the P-level sum dp and the 16-lane trees in the lane kernel's order: model 0 places its states
// on lanes by kStateOfLane0 (see mdqt_internal.hpp), the other models on lane = state
template <int MODEL>
__device__ __forceinline__ double sum_p(const double* Tp) {     // Tp[q] of P state 2 + q
    if constexpr (MODEL == 0) return ((Tp[0] + Tp[2]) + Tp[1]) + Tp[3];   // lanes 0, 3, 4, 7
    return (Tp[0] + Tp[1]) + (Tp[2] + Tp[3]);
}
template <int MODEL>
__device__ __forceinline__ double tree_lanes(const double* vs) {   // vs by state
    double v[16];
#pragma unroll
    for (int l = 0; l < 16; ++l) {
        const int st = MODEL == 0 ? state_of_lane0(l) : l;
        v[l] = st < NS ? vs[st] : 0.;
    }
    return tree16n(v);
}

template <int MODEL>
__global__ __launch_bounds__(256) void k_substeps_r(SubstepArgs a, const FastTab* __restrict__ tab) {
    constexpr const int(&COL)[NS][3] = kFastColM[MODEL];
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.n) return;
    const QTConst& qc = a.qc;
    const FastTab& T = *tab;
    const int S = a.S;
    double P[3], Vv[3], Fv[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        P[c] = a.R[(size_t)c * S + i];
        Vv[c] = a.V[(size_t)c * S + i];
        if (a.nseg > 1) {
            Fv[c] = slot_sum16(a.Fpart + (size_t)c * S + i, (size_t)3 * S, a.nseg);
            a.F[(size_t)c * S + i] = Fv[c];
        } else {
            Fv[c] = a.F[(size_t)c * S + i];
        }
    }
    double tPart = a.tPart[i];
    cxd w[NS + 1];                          // w[NS]: the zero state of model 0's unused slots
    w[NS] = {0., 0.};
    if (a.do_qt) {
#pragma unroll
        for (int k = 0; k < NS; ++k) w[k] = {a.psi[(size_t)(2 * k) * S + i], a.psi[(size_t)(2 * k + 1) * S + i]};
    }
    const double L = a.L, dt = qc.dtQ, DT = 0.5 * dt, DT2 = T.dt2;
    const uint64_t gid = a.gid0 + (uint64_t)i;
    for (int s = 0; s < a.nsub; ++s) {
        if (a.do_step) {
            const bool moving = a.t[s] > 0;
#pragma unroll
            for (int c = 0; c < 3; ++c) {
                P[c] = half_drift(P[c], Vv[c], Fv[c], moving, DT, DT2, L);
                Vv[c] = Vv[c] + dt * Fv[c];
                P[c] = half_drift(P[c], Vv[c], Fv[c], moving, DT, DT2, L);
            }
        }
        if (!a.do_qt) continue;
        const double u = Vv[0] * qc.pv2q + a.expDet[s];
        tPart += qc.dtQ;
        double Tp[4];
#pragma unroll
        for (int q = 0; q < 4; ++q) Tp[q] = nrm2(w[2 + q]) * T.hdp[2 + q];
        const double dp = sum_p<MODEL>(Tp);
        double u1, u2;
        draw_pair(qc, a.U, S, i, gid, a.q0 + (uint64_t)s, 0, u1, u2);
        double kick;
        if (u1 > dp) {
            double kv[NS];
#pragma unroll
            for (int k = 0; k < NS; ++k)
                kv[k] = kick_term(w[k], w[COL[k][0]], w[COL[k][1]], w[COL[k][2]], T.kw[0][k],
                                  T.kw[1][k], T.kw[2][k]);
            kick = sum_p<MODEL>(kv + 2);                 // the kick terms sit on the P lanes
            const double phi = (u * T.cphi) * tPart;
            double sn, cs;
            sincos_q2(phi, kSinCos64, sn, cs);
            cxd md[NS], c2[NS];
#pragma unroll
            for (int k = 0; k < NS; ++k) {
                md[k] = {T.mre[k], fma(T.mi1[k], u, T.mi0[k])};
                c2[k] = {fma(T.dms[k], sn, T.cre[2][k]), fma(T.dmc[k], cs, T.cim[2][k])};
            }
            cxd y[NS + 1], acc[NS];
#pragma unroll
            for (int k = 0; k <= NS; ++k) y[k] = w[k];
#pragma unroll
            for (int stg = 0; stg < 4; ++stg) {
                double dpy = dp;
                if (stg > 0) {
#pragma unroll
                    for (int q = 0; q < 4; ++q) Tp[q] = nrm2(y[2 + q]) * T.hdp[2 + q];
                    dpy = sum_p<MODEL>(Tp);
                }
                const double pref = rsq_nr(1. - dpy);
                cxd ws[NS];
#pragma unroll
                for (int k = 0; k < NS; ++k)
                    ws[k] = row_r(md[k], y[k], cxd{T.cre[0][k], T.cim[0][k]}, y[COL[k][0]],
                                  cxd{T.cre[1][k], T.cim[1][k]}, y[COL[k][1]], c2[k], y[COL[k][2]]);
#pragma unroll
                for (int k = 0; k < NS; ++k) {
                    const cxd d = {fma(pref, ws[k].re, -y[k].re), fma(pref, ws[k].im, -y[k].im)};
                    if (stg == 0) acc[k] = d;
                    else if (stg < 3) acc[k] = {fma(3., d.re, acc[k].re), fma(3., d.im, acc[k].im)};
                    else acc[k] = {acc[k].re + d.re, acc[k].im + d.im};
                    if (stg < 2) y[k] = {fma(0.5, d.re, w[k].re), fma(0.5, d.im, w[k].im)};
                    else if (stg == 2) y[k] = {w[k].re + d.re, w[k].im + d.im};
                }
            }
#pragma unroll
            for (int k = 0; k < NS; ++k) w[k] = {fma(0.125, acc[k].re, w[k].re), fma(0.125, acc[k].im, w[k].im)};
        } else {
            tPart = 0;
            double randDOrS, randDir, rand3, dummy;
            draw_pair(qc, a.U, S, i, gid, a.q0 + (uint64_t)s, 1, randDOrS, randDir);
            draw_pair(qc, a.U, S, i, gid, a.q0 + (uint64_t)s, 2, rand3, dummy);
            (void)dummy;
            const int target = MODEL == 0 ? jump_target(qc, sq(w[2]), sq(w[3]), sq(w[4]), sq(w[5]), u2, randDOrS,
                                                        randDir, rand3, kick)
                                          : jump_target_pump(qc, sq(w[2]), sq(w[3]), sq(w[4]), sq(w[5]), u2,
                                                             randDOrS, randDir, rand3, kick);
#pragma unroll
            for (int k = 0; k < NS; ++k) w[k] = {k == target ? 1. : 0., 0.};
        }
        if (qc.renorm) {                                                    // :706-712
            double nv[NS];
#pragma unroll
            for (int k = 0; k < NS; ++k) nv[k] = nrm2(w[k]);
            const double r = rsq_nr(tree_lanes<MODEL>(nv));
#pragma unroll
            for (int k = 0; k < NS; ++k) w[k] = {w[k].re * r, w[k].im * r};
        }
        Vv[0] = fma(1., kick, Vv[0]);                                       // :705
    }
    const double lo = -0.125 * L, hi = 1.125 * L;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        a.R[(size_t)c * S + i] = P[c];
        a.V[(size_t)c * S + i] = Vv[c];
        if (!(P[c] >= lo && P[c] <= hi)) *a.oor = 1;
    }
    if (a.do_qt) {
        a.tPart[i] = tPart;
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            a.psi[(size_t)(2 * k) * S + i] = w[k].re;
            a.psi[(size_t)(2 * k + 1) * S + i] = w[k].im;
        }
    }
}

// ------------------------------------------------------------------------------------------
// lane per state: one ion per 16-lane group (4 per wave64).  DPPX (model 0): states on lanes by
// kStateOfLane0 and the three coupling slots gathered with DPP moves (lane ^ 2, lane + 8,
// lane ^ 1); lanes 9 / 10 hold the y / z coordinate, every other lane x.  Otherwise (the pumping
// models): lane k = state k, slots gathered through LDS, lanes 12 / 13 hold y / z.  Lanes
// without a state carry zero amplitudes and zero coefficients.  `tab` is indexed by lane.
// ------------------------------------------------------------------------------------------
// dp of model 0's layout: ((T_lane0 + T_lane3) + T_lane4) + T_lane7 = ((T2 + T4) + T3) + T5, in
// every lane — one 64-bit broadcast, then three v_fmac_f64_dpp row_newbcast (the DP ALU takes a
// row_newbcast operand: broadcast and add in one instruction; x * 1 + a is exactly x + a).  `one`
// is 1.0 in a VGPR the compiler cannot see through, so the FMA is kept and the DPP move folds in.
__device__ __forceinline__ double opaque_one() {
    double o = 1.0;
    asm volatile("" : "+v"(o));
    return o;
}
// a + T[lane L of the row] * one as one v_fmac_f64_dpp (the compiler does not fold the 64-bit
// DPP move into the FMA).  DPP read-after-VALU-write hazard: T is also the operand of the
// compiler-emitted broadcast before the first of these, so the write is >= 2 states back.
template <int L>
__device__ __forceinline__ double fmac_bcast(double a, double T, double one) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm("v_fmac_f64_dpp %0, %1, %2 row_newbcast:%3 row_mask:0xf bank_mask:0xf bound_ctrl:1"
        : "+v"(a) : "v"(T), "v"(one), "n"(L));
    return a;
#else
    return fma(T, one, a);
#endif
}
__device__ __forceinline__ double lane_norm16(double v, double one) {
    if (!MDQT_NORM_Q) return lane_tree16(v);
    double a = v + dpp<SHL(1)>(v);                  // lane 2m: v_2m + v_2m+1
    a = a + dpp<SHL(2)>(a);                         // lane 4m: Q_m
    double b = dpp<BCAST(0)>(a);
    b = fmac_bcast<4>(b, a, one);
    b = fmac_bcast<8>(b, a, one);
    return fmac_bcast<12>(b, a, one);
}
__device__ __forceinline__ double lane_sum_p8(double T, double one) {
    double a = dpp<BCAST(0)>(T);
    a = fmac_bcast<3>(a, T, one);
    a = fmac_bcast<4>(a, T, one);
    return fmac_bcast<7>(a, T, one);
}

// the lane kernel's state stores (R, V, F, tPart, psi) write-through, like the force slots
// (mdqt_pairs.hpp MDQT_SLOT_WT): waves that finish early stream their ions out before the last
// wave ends, and the kernel-end L2 write-back has nothing left to do.  A/B at C2 on top of the
// slot stores: QT launch -0.4 us, MD step -0.6 us.  0: plain stores (A/B builds).
#ifndef MDQT_QT_WT
#define MDQT_QT_WT 1
#endif
__device__ __forceinline__ void qt_store(double* p, double v) {
    if constexpr (MDQT_QT_WT) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}

#if defined(MDQT_EXPT_QTSTAMPS)
// diagnostic build only: per-wave s_memtime at entry, loop start, loop end, exit + s_memrealtime
// at entry and exit, s_memtime after the force-slot loads (6), after the prologue's loads are
// issued (9) and after the Philox draws (8), and the number of substeps in which an ion of the
// wave jumped (7) (tools/qt_stamps.py)
__device__ unsigned long long g_qt_stamps[16 * 4096];
#define QT_STAMP(slot, v) (st_[slot] = (v))
#define QT_JCOUNT(c) (st_[7] += (__builtin_amdgcn_ballot_w64(c) != 0))
#else
#define QT_STAMP(slot, v) ((void)0)
#define QT_JCOUNT(c) ((void)0)
#endif

#if defined(MDQT_EXPT_MDSTAMPS)
// diagnostic build only (k_md_step): per-workgroup s_memrealtime at entry and exit (+ after the
// wait, QT workgroups)
__device__ unsigned long long g_md_stamps[4 * 4096];
#endif

#ifndef MDQT_LANE_WPE
#define MDQT_LANE_WPE 0
#endif
#if MDQT_LANE_WPE > 0
#define LANE_WPE_ATTR __attribute__((amdgpu_waves_per_eu(MDQT_LANE_WPE, MDQT_LANE_WPE)))
#else
#define LANE_WPE_ATTR
#endif
// FAST: the production launch — step + qstep (do_step, do_qt), every substep with t > 0 (all but
// the simulation's first launch), F from the force slots (or F itself when nseg == 1), no arrival
// wait: step_R's
// non-moving branch (:360), the last substep's no-drift select and the other paths' loads and
// branches are compiled out (straight-line prologue: one memory round trip)
// FUSED (with FAST; the QT workgroups of k_md_step): the force partials of this launch's own
// tile pairs are read after the arrival count of the ions' tile is complete, with L1-bypassing
// loads (the tile pairs' slot stores are write-through: MI355X_MICROARCH.md, hand-off forms)
// IM01 (with FAST): the static coupling slots 0 and 1 are purely imaginary (QTConst::im01), their
// real-part FMAs are dropped.  EDZ: every expDetuning of the launch is 0 (u = vx pv2q).  The
// production model-0 launch is k_substeps_lanes_im<true, true> (FAST + IM01 + EDZ).
// NORN: reNormalizewvFns is off (the reference's default, SpeedUp:74) — the renormalisation and
// its uniform branch compiled out, so one substep's tail and the next one's head share a basic block
template <bool DPPX, bool FAST, bool FUSED, bool IM01 = false, bool EDZ = false, bool NORN = false>
__device__ __forceinline__ void lane_substeps(const SubstepArgs& a, const FastTab* __restrict__ tab, int blk) {
#if defined(MDQT_EXPT_QTSTAMPS)
    unsigned long long st_[16] = {};
#endif
    QT_STAMP(0, __builtin_amdgcn_s_memtime());
    QT_STAMP(4, __builtin_amdgcn_s_memrealtime());
    const int k = threadIdx.x & 15;
    const int grp = threadIdx.x >> 4;
    const int iraw = kRows == 4 ? blk * (kLaneWG / 16) + grp
                                : (blk * (kLaneWG / 64) + (grp >> 2)) * kRows + ((grp & 3) % kRows);
    const bool store = iraw < a.n && (kRows == 4 || (grp & 3) < kRows);
    const int i = store ? iraw : a.n - 1;             // idle groups shadow the last ion
    const QTConst& qc = a.qc;
    const int S = a.S;
    const int st = DPPX ? state_of_lane0(k) : k;      // >= NS: no state on this lane
    const int cy = DPPX ? 9 : 12, cz = DPPX ? 10 : 13;
    const int c = (k == cy) ? 1 : (k == cz) ? 2 : 0;
    const bool owner = (k == 0) || (k == cy) || (k == cz);   // stores coordinate c
    const int base = threadIdx.x & ~15;
    const int l0 = base + tab->col[0][k], l1 = base + tab->col[1][k], l2 = base + tab->col[2][k];
    const cxd c0 = {tab->cre[0][k], tab->cim[0][k]}, c1 = {tab->cre[1][k], tab->cim[1][k]};
    const double c2re = tab->cre[2][k], c2im = tab->cim[2][k], dms = tab->dms[k], dmc = tab->dmc[k];
    const double mre = tab->mre[k], mi0 = tab->mi0[k], mi1 = tab->mi1[k], hdp = tab->hdp[k];
    const double kw0 = tab->kw[0][k], kw1 = tab->kw[1][k], kw2 = tab->kw[2][k];
    const double cphi = tab->cphi, DT2 = tab->dt2;
    const double kmask = (c == 0) ? 1. : 0.;
    const double one = opaque_one();
    // Prologue: every load is issued before any is consumed (one memory round trip), and the
    // lane-parallel Philox draws below run while they are in flight.
    double p = a.R[(size_t)c * S + i], v = a.V[(size_t)c * S + i], f;
    double tPart = a.tPart[i];
    cxd w = {0., 0.};
    if ((FAST || a.do_qt) && st < NS) w = {a.psi[(size_t)(2 * st) * S + i], a.psi[(size_t)(2 * st + 1) * S + i]};
    const int nseg = a.nseg;
    // F: the canonical slot_sum16 distributed over the ion's 16 lanes — lane k forms the strided
    // partial q_k of all three components (its loads issued together, 4 slots per round), the
    // DPP tree combines them in slot_sum16's order
    double qf[3] = {0., 0., 0.};
    // overlapped MD step (a.arrive): the partials are read after the arrival wait below, with
    // L1-bypassing loads; otherwise right here, with the other prologue loads
    auto slot_round = [&](int s0, double (*t)[3], bool sc1) {   // slots s0, s0 + 16, + 32, + 48
        // FAST with nseg == 1 (F already summed): slot 0 is F itself, the other lanes add zeros
        const double* base_p = (FAST && nseg == 1 ? (const double*)a.F : a.Fpart) + i;
        const size_t plane = (size_t)3 * S;
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int sl = s0 + 16 * u;
#pragma unroll
            for (int cc = 0; cc < 3; ++cc) {
                if (FAST) {   // unconditional loads (clamped slot, in range), the select at the sum:
                              // no branch around the load, so nothing forces an early wait on it
                    const double* q = base_p + (size_t)min(sl, nseg - 1) * plane + (size_t)cc * S;
#if defined(MDQT_EXPT_NTSLOT)
                    const double x = sc1 ? __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT)
                                         : __builtin_nontemporal_load(q);   // A/B: read-once slots as nt loads
#else
                    const double x = sc1 ? __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *q;
#endif
                    t[u][cc] = sl < nseg ? x : 0.;
                } else {
                    const double* q = base_p + (size_t)sl * plane + (size_t)cc * S;
                    t[u][cc] = sl < nseg ? (sc1 ? __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : *q)
                                         : 0.;
                }
            }
        }
    };
    auto slot_add = [&](double (*t)[3]) {
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int cc = 0; cc < 3; ++cc) qf[cc] = qf[cc] + t[u][cc];
    };
    auto slot_partials = [&](bool sc1) {
        for (int s0 = k; s0 < nseg; s0 += 64) {
            double t[4][3];
            slot_round(s0, t, sc1);
            slot_add(t);
        }
    };
    // FAST: the first round's loads stay in flight across the Philox draws below; summed after
    double t0[4][3];
    if (FAST) {
        if (!FUSED) slot_round(k, t0, false);
    } else if (nseg > 1) {
        if (!a.arrive) slot_partials(false);
    } else {
        f = a.F[(size_t)c * S + i];
    }
    QT_STAMP(9, __builtin_amdgcn_s_memtime());
    const double L = a.L, dt = qc.dtQ, DT = 0.5 * dt;
    // the substep loop's tPart step and Doppler factor held in VGPRs: with every SGPR taken the
    // compiler otherwise re-loads them from the kernel arguments inside the loop, and the
    // s_waitcnt on that scalar load stalls every substep
    double dtq_v = qc.dtQ, pv2q_v = qc.pv2q;
    asm volatile("" : "+v"(dtq_v), "+v"(pv2q_v));
    const uint64_t gid = a.gid0 + (uint64_t)i;
    // per-substep constants out of kernel-argument loads inside the substep loop (a scalar load
    // indexed by the substep waits ~100+ cycles in every iteration): the moving flags as a bit
    // mask, expDetuning(t) of every substep in an LDS row (one broadcast read per substep, issued
    // with the uniforms; it replaces a readlane and its scalar branches in every iteration)
    const uint32_t movmask = a.movmask;
    __shared__ double edt[MAXSUB];
    // (loaded here, written to LDS after the force sum below: an LDS write of a loaded value waits
    // for every load issued before it, which would stall the Philox draws behind the slot loads)
    const double edv = (threadIdx.x < MAXSUB && a.expdet_zero == 0 && (int)threadIdx.x < a.nsub)
                           ? a.expDet[threadIdx.x] : 0.;
    // the coupling phase's e^(2 pi i j / 64) table (sincos_tab) in LDS, written with edt below
    __shared__ double sct[128];
    const double sctv = (MDQT_QT_SCTAB && threadIdx.x < 128) ? kSinCos64[threadIdx.x] : 0.;
    // u1, u2 of every substep of the launch staged in LDS: Philox draws computed lane-parallel
    // (lane k: substeps k, k + 16), or the rng_mode 0 uniforms of the single substep
    __shared__ double su[kLaneWG / 16][MAXSUB][2];
    if (FAST || a.do_qt) {
        if (a.U) {
            if (k == 0) { su[grp][0][0] = a.U[i]; su[grp][0][1] = a.U[(size_t)S + i]; }
        } else {
            for (int s = k; s < a.nsub; s += 16) {
                double x0, x1;
                philox_pair(qc, gid, a.q0 + (uint64_t)s, 0, x0, x1);
                su[grp][s][0] = x0;
                su[grp][s][1] = x1;
            }
        }
    }
    QT_STAMP(8, __builtin_amdgcn_s_memtime());
    if (!FAST && a.arrive) {                          // wait for the concurrent force launch
        if (threadIdx.x == 0) {
            int it = 0;
            const unsigned long long* cnt = a.arrive + (blk * (kLaneWG / 16)) / 64;   // the ions' tile
            while (__hip_atomic_load(cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < a.arrive_target) {
                for (int z = 0; z < a.arrive_sleep; ++z) __builtin_amdgcn_s_sleep(1);
                if (++it > (1 << 21)) { *a.spin_err = 1; break; }   // bounded: never hang the GPU
            }
        }
        __syncthreads();                              // thread 0's acquire, then the workgroup's loads
        __atomic_thread_fence(__ATOMIC_ACQUIRE);       // (workgroup fence: no early slot load)
        if (nseg > 1) slot_partials(true);
    }
    if (FUSED) {                                      // this launch's tile pairs of the ions' tile
        if (threadIdx.x == 0) {
            const unsigned long long* cnt = a.arrive + (blk * (kLaneWG / 16)) / 64;
            int it = 0;
            while (__hip_atomic_load(cnt, __ATOMIC_ACQUIRE, __HIP_MEMORY_SCOPE_AGENT) < a.arrive_target) {
                __builtin_amdgcn_s_sleep(2);
                if (++it > (1 << 22)) { *a.spin_err = 1; break; }   // bounded: never hang the GPU
            }
        }
        __syncthreads();
        __atomic_thread_fence(__ATOMIC_ACQUIRE);
#if defined(MDQT_EXPT_MDSTAMPS)
        if (threadIdx.x == 0 && blockIdx.x < 4096) g_md_stamps[4 * blockIdx.x + 2] = __builtin_amdgcn_s_memrealtime();
#endif
        slot_round(k, t0, true);
    }
    if (FAST) {
        slot_add(t0);
        for (int s0 = k + 64; s0 < nseg; s0 += 64) {
            double t[4][3];
            slot_round(s0, t, FUSED);
            slot_add(t);
        }
    }
    QT_STAMP(6, __builtin_amdgcn_s_memtime());
    if (FAST || nseg > 1) {
        const double fx = lane_tree16(qf[0]), fy = lane_tree16(qf[1]), fz = lane_tree16(qf[2]);
        f = c == 0 ? fx : c == 1 ? fy : fz;
        if (store && owner) qt_store(&a.F[(size_t)c * S + i], f);
    }
    if (threadIdx.x < MAXSUB) edt[threadIdx.x] = edv;
    if (MDQT_QT_SCTAB && threadIdx.x < 128) sct[threadIdx.x] = sctv;
    __syncthreads();
    __shared__ double2 xg[DPPX ? 1 : kLaneWG];
    auto exchange = [&](cxd y, cxd& y0, cxd& y1, cxd& y2) {
        if constexpr (DPPX) {
            y0 = {dpp<QP_XOR2>(y.re), dpp<QP_XOR2>(y.im)};
            y1 = {dpp<ROR(8)>(y.re), dpp<ROR(8)>(y.im)};
            y2 = {dpp<QP_XOR1>(y.re), dpp<QP_XOR1>(y.im)};
            return;
        }
        wave_sync();
        xg[threadIdx.x] = make_double2(y.re, y.im);
        wave_sync();
        const double2 t0 = xg[l0], t1 = xg[l1], t2 = xg[l2];
        y0 = {t0.x, t0.y}; y1 = {t1.x, t1.y}; y2 = {t2.x, t2.y};
    };
    auto drift = [&](double& pp, double& vv, int sub) {   // step(): step_R, step_V, step_R (:418-430)
        const bool moving = FAST || ((movmask >> sub) & 1u);
        pp = half_drift(pp, vv, f, moving, DT, DT2, L);
        vv = vv + dt * f;                             // step_V(dt) :398-409
        pp = half_drift(pp, vv, f, moving, DT, DT2, L);
    };
    QT_STAMP(1, __builtin_amdgcn_s_memtime());
    if (!FAST && !a.do_qt) {
        if (a.do_step)
            for (int s = 0; s < a.nsub; ++s) drift(p, v, s);
    } else {
        // Software-pipelined substeps: once substep s has its kick, the drift of substep s + 1
        // and the sin / cos of its coupling phase (:508) depend on nothing else of substep s, so
        // they are evaluated before s's Runge-Kutta stages and overlap them.  Same operations on
        // the same values as the plain order: bit-identical.
        if (FAST || a.do_step) drift(p, v, 0);
        double pre_p = p, pre_v = v;                  // FAST: the state after the last substep
        double sn, cs;
        // (EDZ: every expDet of the launch is 0 — fracOfSig = 0, the default — so u = vx pv2q: the
        // + 0 and its LDS read dropped; the same values up to the sign of an exact zero)
        double u = EDZ ? v * pv2q_v : v * pv2q_v + edt[0];     // vx on every state lane (carried: the
        double tn = tPart + dtq_v;                    // next substep's is formed with its phase); tn:
        sincos_q2((u * cphi) * tn, sct, sn, cs);      // the next substep's tPart, formed once
#if defined(MDQT_EXPT_PHASEROT)
        double phi_c = (u * cphi) * tn;
#endif
#ifndef MDQT_QT_UNROLL
#define MDQT_QT_UNROLL 2
#endif
#ifndef MDQT_PHASE_BOUND
#define MDQT_PHASE_BOUND 1
#endif
        // Wave-uniform bound on every coupling phase of the launch (production instance): |v| grows
        // by at most |dt f| + kickmax per substep and tPart by dtQ, so when the bound on |phi| is
        // below 2^19 the per-substep |phi| >= 2^20 library fallback cannot trigger and is left out
        // of the loop (it would split every substep's tail from the next one's head into separate
        // basic blocks); otherwise the loop keeps it.  The same values either way.
        bool phase_small = false;
        if constexpr (FAST && EDZ && DPPX && MDQT_PHASE_BOUND) {
            const double vb = fabs(v) + (double)(a.nsub + 1) * (fabs(dt * f) + qc.kickmax);
            const double tb = fabs(tPart) + (double)(a.nsub + 1) * dtq_v;
            const double pb = ((vb * fabs(pv2q_v)) * fabs(cphi)) * tb;
            phase_small = __builtin_amdgcn_ballot_w64(!(pb < 524288.)) == 0;
        }
        auto substep = [&](int s, auto chk) {
            tPart = tn;                               // tPart += dtQ (formed in the last next_phase)
            const double dp = DPPX ? lane_sum_p8(nrm2(w) * hdp, one) : lane_sum_p(nrm2(w) * hdp);
            const double u1 = su[grp][s][0], u2 = su[grp][s][1];
            cxd w0, w1, w2;
            exchange(w, w0, w1, w2);
            double kick;
#if defined(MDQT_EXPT_NOJUMP)
            const bool nojump = true;                 // timing-only diagnostic build: no jumps
            (void)u1;
#else
            const bool nojump = u1 > dp;
#endif
            QT_JCOUNT(!nojump);
            // substep s + 1's drift and phase, placed in the same basic block as the work they
            // overlap (straight-line: the last substep computes a harmless extra value, the
            // |phi| >= 2^20 library fallback is applied afterwards)
            double vn, pn, un, phin, snn, csn;
            auto next_phase = [&]() {
                vn = fma(kmask, kick, v);             // :705 (x lanes)
                pn = p;
                const int s1 = s + 1 < a.nsub ? s + 1 : s;
                double pd = pn, vd = vn;
                drift(pd, vd, s1);
                if constexpr (FAST) {                 // always advance; the launch keeps the state
                    pre_p = pn;                       // before the last substep's extra drift
                    pre_v = vn;
                    pn = pd;
                    vn = vd;
                } else {
                    const bool adv = a.do_step && s + 1 < a.nsub;   // no drift after the last substep
                    pn = adv ? pd : pn;
                    vn = adv ? vd : vn;
                }
                un = EDZ ? vn * pv2q_v : vn * pv2q_v + edt[s1];
                tn = tPart + dtq_v;
                phin = (un * cphi) * tn;
#if defined(MDQT_EXPT_PHASEROT)
                {   // timing-only diagnostic: e^(i phin) = e^(i phi) e^(i dphi), short Taylor series of
                    // dphi without range reduction (wrong for large dphi and after a jump: NOT a product form)
                    const double dph = phin - phi_c, z = dph * dph;
                    const double sd = dph * fma(z, fma(z, fma(z, -1.984126984126984e-04, 8.333333333333333e-03),
                                                       -1.666666666666667e-01), 1.0);
                    const double cd = fma(z, fma(z, fma(z, fma(z, 2.48015873015873e-05, -1.388888888888889e-03),
                                                        4.166666666666666e-02), -0.5), 1.0);
                    snn = fma(sn, cd, cs * sd);
                    csn = fma(cs, cd, -(sn * sd));
                    phi_c = phin;
                }
#else
                if (MDQT_QT_SCTAB) sincos_tab(phin, sct, snn, csn);
                else sincos_fast(phin, snn, csn);
#endif
            };
            if (nojump) {
                {                                 // kick terms on the P lanes (host table)
                    const double kt = kick_term(w, w0, w1, w2, kw0, kw1, kw2);
                    kick = DPPX ? lane_sum_p8(kt, one) : lane_sum_p(kt);
                }
                next_phase();
                const cxd md = {mre, fma(mi1, u, mi0)};
                const cxd c2 = {fma(dms, sn, c2re), fma(dmc, cs, c2im)};
                cxd y = w, acc = {0., 0.};
                cxd y0 = w0, y1 = w1, y2 = w2;
#pragma unroll
                for (int stg = 0; stg < 4; ++stg) {
                    double dpy = dp;
                    if (stg > 0) {
                        dpy = DPPX ? lane_sum_p8(nrm2(y) * hdp, one) : lane_sum_p(nrm2(y) * hdp);
                        exchange(y, y0, y1, y2);
                    }
                    const double pref = rsq_nr(1. - dpy);
                    const cxd ws = IM01 ? row_r_im01(md, y, c0.im, y0, c1.im, y1, c2, y2)
                                        : row_r(md, y, c0, y0, c1, y1, c2, y2);
                    const cxd d = {fma(pref, ws.re, -y.re), fma(pref, ws.im, -y.im)};
                    if (stg == 0) acc = d;
                    else if (stg < 3) acc = {fma(3., d.re, acc.re), fma(3., d.im, acc.im)};
                    else acc = {acc.re + d.re, acc.im + d.im};
                    if (stg < 2) y = {fma(0.5, d.re, w.re), fma(0.5, d.im, w.im)};
                    else if (stg == 2) y = {w.re + d.re, w.im + d.im};
                }
                w = {fma(0.125, acc.re, w.re), fma(0.125, acc.im, w.im)};
            } else {                                  // quantum jump (:573-703)
                tPart = 0;
                const double nk = sq(w);
                double n3, n4, n5, n6;                    // |w|^2 of the P states 2..5
                if constexpr (DPPX) {
                    n3 = dpp<BCAST(0)>(nk); n4 = dpp<BCAST(4)>(nk); n5 = dpp<BCAST(3)>(nk); n6 = dpp<BCAST(7)>(nk);
                } else {
                    n3 = dpp<BCAST(2)>(nk); n4 = dpp<BCAST(3)>(nk); n5 = dpp<BCAST(4)>(nk); n6 = dpp<BCAST(5)>(nk);
                }
                double randDOrS, randDir, rand3, dummy;
                if (a.U) {
                    draw_pair(qc, a.U, S, i, gid, a.q0 + (uint64_t)s, 1, randDOrS, randDir);
                    draw_pair(qc, a.U, S, i, gid, a.q0 + (uint64_t)s, 2, rand3, dummy);
                    (void)dummy;
                } else {                              // both pairs in one Philox evaluation: lanes 0-7
                    double x0, x1;                    // draw pair 1, lanes 8-15 pair 2 (the whole
                    philox_pair(qc, gid, a.q0 + (uint64_t)s, k < 8 ? 1 : 2, x0, x1);   // group is active)
                    randDOrS = dpp<BCAST(0)>(x0);
                    randDir = dpp<BCAST(0)>(x1);
                    rand3 = dpp<BCAST(8)>(x0);
                }
                const int target = (DPPX || qc.model == 0)   // DPPX: model 0
                                       ? jump_target(qc, n3, n4, n5, n6, u2, randDOrS, randDir, rand3, kick)
                                       : jump_target_pump(qc, n3, n4, n5, n6, u2, randDOrS, randDir, rand3, kick);
                w = {st == target ? 1. : 0., 0.};
                next_phase();
            }
            if constexpr (decltype(chk)::value)
                if (!(fabs(phin) < 1048576.)) sincos(phin, &snn, &csn);
            if (!NORN && qc.renorm) w = [&] {             // :706-712
                const double r = rsq_nr(lane_norm16(nrm2(w), one));
                return cxd{w.re * r, w.im * r};
            }();
            v = vn;
            p = pn;
            u = un;
            sn = snn;
            cs = csn;
        };
        auto loop = [&](auto chk) {
            if (MDQT_QT_UNROLL == 2) {                // two substeps per iteration (register copies)
                int s = 0;
                for (; s + 1 < a.nsub; s += 2) {
                    substep(s, chk);
                    substep(s + 1, chk);
                }
                if (s < a.nsub) substep(s, chk);
            } else {
                for (int s = 0; s < a.nsub; ++s) substep(s, chk);
            }
        };
        if (phase_small) loop(std::false_type{});
        else loop(std::true_type{});
        if constexpr (FAST) {
            p = pre_p;
            v = pre_v;
        }
    }
    QT_STAMP(2, __builtin_amdgcn_s_memtime());
    if (store) {
        if (owner) {
            qt_store(&a.R[(size_t)c * S + i], p);
            qt_store(&a.V[(size_t)c * S + i], v);
            if (!(p >= -0.125 * L && p <= 1.125 * L)) *a.oor = 1;
        }
        if (FAST || a.do_qt) {
            if (k == 0) qt_store(&a.tPart[i], tPart);
            if (st < NS) {
                qt_store(&a.psi[(size_t)(2 * st) * S + i], w.re);
                qt_store(&a.psi[(size_t)(2 * st + 1) * S + i], w.im);
            }
        }
    }
#if defined(MDQT_EXPT_QTSTAMPS)
    __builtin_amdgcn_s_waitcnt(0);
    st_[3] = __builtin_amdgcn_s_memtime();
    st_[5] = __builtin_amdgcn_s_memrealtime();
    const int wv = (int)(blk * (kLaneWG / 64) + (threadIdx.x >> 6));
    if ((threadIdx.x & 63) < 16 && wv < 4096) {             // vector stores, one slot per lane
        const int q = threadIdx.x & 63;
        unsigned long long v = st_[0];
#pragma unroll
        for (int m = 1; m < 16; ++m) v = (q == m) ? st_[m] : v;
        g_qt_stamps[16 * wv + q] = v;
    }
#endif
}

template <bool DPPX, bool FAST>
__global__ __launch_bounds__(256) LANE_WPE_ATTR void k_substeps_lanes_r(SubstepArgs a, const FastTab* __restrict__ tab) {
    lane_substeps<DPPX, FAST, false>(a, tab, blockIdx.x);
}
// the FAST launch when QTConst::im01 (the production model-0 case); EDZ: expdet_zero
template <bool DPPX, bool EDZ, bool NORN = false>
__global__ __launch_bounds__(256) LANE_WPE_ATTR void k_substeps_lanes_im(SubstepArgs a, const FastTab* __restrict__ tab) {
    lane_substeps<DPPX, true, false, true, EDZ, NORN>(a, tab, blockIdx.x);
}

// ------------------------------------------------------------------------------------------
// k_md_step: one MD step of one system (world 1, Newton-3 tiles, the lane QT kernel's FAST
// instance) in ONE launch — forces() (SpeedUp:192-236) then the interval's fused step(); qstep();
// substeps (:1376-1377).  Workgroups [0, npairs) are the tile pairs of k_pairs_n3 (same body,
// write-through slot stores, one arrival per tile whose rows they wrote); workgroups npairs.. are
// the lane kernel's 16-ion groups, which do their prologue (loads, Philox draws) while the force
// workgroups run and wait for the arrival count of their ions' tile before reading the slots.
// Workgroups are dispatched in index order, so every force workgroup is placed before any QT
// workgroup: the waits cannot starve a force workgroup of a slot.  Same operations on the same
// values as the two launches: bit-identical (tests/test_gpu_parity.py).  Saves the QT launch's
// dispatch and hides its prologue behind the force kernel's tail.
// ------------------------------------------------------------------------------------------
static_assert(kLaneWG == 64 * N3W, "k_md_step: one workgroup size for both parts");
#if defined(MDQT_EXPT_MDSTAMPS)
extern "C" int mdqt_expt_md_stamps(unsigned long long* out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_md_stamps), sizeof(unsigned long long) * 4 * n) == hipSuccess ? 0 : -1;
}
#define MD_STAMP(slot) \
    do { if (threadIdx.x == 0 && blockIdx.x < 4096) g_md_stamps[4 * blockIdx.x + (slot)] = __builtin_amdgcn_s_memrealtime(); } while (0)
#else
#define MD_STAMP(slot) ((void)0)
#endif
template <bool DPPX, int VARIANT>
__global__ __launch_bounds__(256) void k_md_step(N3Args f, SubstepArgs a, const FastTab* __restrict__ tab) {
    MD_STAMP(0);
    if ((int)blockIdx.x < f.npairs) {
        __shared__ double pj[3][128];
        __shared__ double accj[N3W][3][128];
        __shared__ double ia[N3W][3][64];
        __shared__ double mj[128];
        __shared__ double etab[64];
        stage_exp_tab(etab);
        const int2 IJ = f.pairs[blockIdx.x];
        const PairC c = {f.L, f.micT, f.micGuard, f.Rcut, f.lDeb, f.invlDeb, 1. / f.L, f.rc2, etab};
        const bool rag = (f.N & 63) && IJ.y == f.ntiles - 1;
        if (rag) n3_tile<VARIANT, false, true, true>(f, c, IJ.x, IJ.y, pj, accj, mj, ia);
        else n3_tile<VARIANT, false, false, true>(f, c, IJ.x, IJ.y, pj, accj, mj, ia);
        MD_STAMP(1);
        return;
    }
    lane_substeps<DPPX, true, true>(a, tab, (int)blockIdx.x - f.npairs);
    MD_STAMP(1);
}

hipError_t launch_md_step(const N3Args& f, const SubstepArgs& a, const FastTab* tab, int variant, hipStream_t s,
                          hipEvent_t ev0, hipEvent_t ev1) {
    if (a.n <= 0 || f.npairs <= 0 || a.nsub <= 0 || a.nsub > MAXSUB || !a.arrive || !f.arrive || f.guard || kRows != 4)
        return hipErrorInvalidValue;
    if (a.qc.model < 0 || a.qc.model >= NMODELS || variant < 0 || variant > 1) return hipErrorInvalidValue;
    const dim3 gl(f.npairs + (a.n + kLaneWG / 16 - 1) / (kLaneWG / 16)), bl(kLaneWG);
    const FastTab* lt = tab + 1;                      // by lane
    if (a.qc.model == 0) {
        if (variant == 1) launch_timed(k_md_step<true, 1>, gl, bl, s, ev0, ev1, f, a, lt);
        else launch_timed(k_md_step<true, 0>, gl, bl, s, ev0, ev1, f, a, lt);
    } else {
        if (variant == 1) launch_timed(k_md_step<false, 1>, gl, bl, s, ev0, ev1, f, a, lt);
        else launch_timed(k_md_step<false, 0>, gl, bl, s, ev0, ev1, f, a, lt);
    }
    return hipGetLastError();
}

#if defined(MDQT_EXPT_QTSTAMPS)
extern "C" int mdqt_expt_qt_stamps(unsigned long long* out, int nwaves) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_qt_stamps), sizeof(unsigned long long) * 16 * nwaves) == hipSuccess ? 0 : -1;
}
#endif

hipError_t launch_substeps_r(const SubstepArgs& a, const FastTab* tab, int mode, hipStream_t s, hipEvent_t ev0,
                             hipEvent_t ev1, int* instance) {
    if (a.n <= 0 || a.nsub <= 0) return hipSuccess;
    if (a.nsub > MAXSUB) return hipErrorInvalidValue;
    if (mode == 0) mode = (a.n < kLaneKernelMaxIons) ? 2 : 1;
    if (a.qc.model < 0 || a.qc.model >= NMODELS) return hipErrorInvalidValue;
    const dim3 gl((a.n + kLaneIons - 1) / kLaneIons), bl(kLaneWG), gt((a.n + 255) / 256), b(256);
    int inst = QTK_THREAD_R + a.qc.model;
    if (mode == 2) {
        const uint64_t all = (1ull << a.nsub) - 1;
        const bool allmove = a.do_step && a.do_qt && a.nseg >= 1 && !a.arrive && (a.movmask & all) == all;
#ifndef MDQT_IM01
#define MDQT_IM01 1
#endif
#ifndef MDQT_EDZ
#define MDQT_EDZ 1
#endif
#ifndef MDQT_NORN
#define MDQT_NORN 1
#endif
        if (a.qc.model == 0) {
            if (allmove && a.qc.im01 && MDQT_IM01) {
                if (a.expdet_zero && MDQT_EDZ && !a.qc.renorm && MDQT_NORN) {   // the production launch
                    launch_timed(k_substeps_lanes_im<true, true, true>, gl, bl, s, ev0, ev1, a, tab + 1);
                    inst = QTK_LANES_IM_EDZ;
                } else if (a.expdet_zero && MDQT_EDZ) {
                    launch_timed(k_substeps_lanes_im<true, true>, gl, bl, s, ev0, ev1, a, tab + 1);
                    inst = QTK_LANES_IM_EDZ_RN;
                } else {
                    launch_timed(k_substeps_lanes_im<true, false>, gl, bl, s, ev0, ev1, a, tab + 1);
                    inst = QTK_LANES_IM;
                }
            } else if (allmove) {
                launch_timed(k_substeps_lanes_r<true, true>, gl, bl, s, ev0, ev1, a, tab + 1);
                inst = QTK_LANES_R_FAST;
            } else {
                launch_timed(k_substeps_lanes_r<true, false>, gl, bl, s, ev0, ev1, a, tab + 1);
                inst = QTK_LANES_R;
            }
        } else {
            if (allmove) {
                launch_timed(k_substeps_lanes_r<false, true>, gl, bl, s, ev0, ev1, a, tab + 1);
                inst = QTK_LANES_R_PUMP_FAST;
            } else {
                launch_timed(k_substeps_lanes_r<false, false>, gl, bl, s, ev0, ev1, a, tab + 1);
                inst = QTK_LANES_R_PUMP;
            }
        }
    }
    else if (a.qc.model == 0) launch_timed(k_substeps_r<0>, gt, b, s, ev0, ev1, a, tab);
    else if (a.qc.model == 1) launch_timed(k_substeps_r<1>, gt, b, s, ev0, ev1, a, tab);
    else if (a.qc.model == 2) launch_timed(k_substeps_r<2>, gt, b, s, ev0, ev1, a, tab);
    else launch_timed(k_substeps_r<3>, gt, b, s, ev0, ev1, a, tab);
    if (instance) *instance = inst;
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// spin-up tagging after the pump window: measureSpinUps (randomFrozenStartTag408Linear.cpp:600,
// randomFrozenStartTag422Linear.cpp:568) = tagParticles (MonteCarloFollowedByQTTagging408Linear.cpp
// :1022).  Draws: Philox (ion, qstep index, draws 6 and 7) for rand and rand2/rand3.
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_tag_spin_up(const double* __restrict__ psi, int n, int S, uint64_t gid0,
                                                     uint64_t q, QTConst qc, int* __restrict__ tags) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    double nr[5];
#pragma unroll
    for (int k = 0; k < 5; ++k) {
        const double re = psi[(size_t)(2 * k) * S + i], im = psi[(size_t)(2 * k + 1) * S + i];
        nr[k] = re * re + im * im;                                   // std::norm
    }
    double rnd, r2;
    philox_pair(qc, gid0 + (uint64_t)i, q, 3, rnd, r2);
    int up;
    if (qc.model == 3) {                                             // 422 (:592-631)
        if (rnd < nr[0]) up = 1;
        else if (rnd < nr[0] + nr[2]) up = r2 < 1. / 3;
        else if (rnd < nr[0] + nr[2] + nr[3]) up = r2 < 2. / 3;
        else up = 0;
    } else {                                                         // 408 (:600-640)
        if (rnd < nr[0] + nr[2]) up = 1;
        else if (rnd < nr[0] + nr[2] + nr[3]) up = r2 < 2. / 3;
        else if (rnd < nr[0] + nr[2] + nr[3] + nr[4]) up = r2 < 1. / 3;
        else up = 0;
    }
    tags[i] = up;
}

hipError_t launch_tag_spin_up(const double* psi, int n, int S, uint64_t gid0, uint64_t q, const QTConst& qc,
                              int* tags, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_tag_spin_up, dim3((n + 255) / 256), dim3(256), 0, s, psi, n, S, gid0, q, qc, tags);
    return hipGetLastError();
}

}  // namespace mdqt
