// Pair terms of forces() (SpeedUp:192-236) and the Newton-3 tile-pair body, shared by the force
// kernels (mdqt_forces.hip) and the fused MD-step kernel (mdqt_qtfast.hip).
#pragma once
#include "mdqt_internal.hpp"

#include <math.h>

namespace mdqt {

struct PairC {
    double L, T, G, Rcut, lDeb, invlDeb, invL;
    double rc2;         // VARIANT 2: pair kept iff r2 < rc2 (= sqrt(r2) < Rcut exactly)
    const double* etab; // the Newton-3 kernels' 2^(j/64) table in LDS (pair_ft_cut, MDQT_EXP_TAB)
    // the tile kernel's box-scaled form (MDQT_N3_SCALED, n3_tile): positions s = x / L, so the minimum
    // image is ds - rint(ds); sA = 1/L^2, sB = 1/(lDeb L), sT = 64 (-log2 e) L / lDeb
    double sA, sB, sT;
};

// 2^t of the Newton-3 kernels' exact pair form by a 64-entry table (round 3, MDQT_EXP_TAB):
// t64 = 64 t (the multiplier scaled by 64: exact), m = rint(t64), g = t64 - m (exact, |g| <= 1/2),
// 2^t = 2^(m >> 6) 2^((m & 63)/64) 2^(g/64) with the table entry correctly rounded (60-digit decimal
// arithmetic) and 2^(g/64) = e^(g ln2/64) by its degree-5 Taylor series (|g ln2/64| <= 0.0055:
// truncation 3.5e-17); <= 2 ulp.  Five FMAs instead of eleven for three integer operations and one
// LDS read; the cutoff folded into the exponent as in exp2_neg_cut.
// (MDQT_EXP_TAB: mdqt_internal.hpp, where the engine's mid-tier radius sees it too)
static __constant__ const double kExp2Tab64[64] = {
    0x1.0000000000000p+0, 0x1.02c9a3e778061p+0, 0x1.059b0d3158574p+0, 0x1.0874518759bc8p+0,
    0x1.0b5586cf9890fp+0, 0x1.0e3ec32d3d1a2p+0, 0x1.11301d0125b51p+0, 0x1.1429aaea92de0p+0,
    0x1.172b83c7d517bp+0, 0x1.1a35beb6fcb75p+0, 0x1.1d4873168b9aap+0, 0x1.2063b88628cd6p+0,
    0x1.2387a6e756238p+0, 0x1.26b4565e27cddp+0, 0x1.29e9df51fdee1p+0, 0x1.2d285a6e4030bp+0,
    0x1.306fe0a31b715p+0, 0x1.33c08b26416ffp+0, 0x1.371a7373aa9cbp+0, 0x1.3a7db34e59ff7p+0,
    0x1.3dea64c123422p+0, 0x1.4160a21f72e2ap+0, 0x1.44e086061892dp+0, 0x1.486a2b5c13cd0p+0,
    0x1.4bfdad5362a27p+0, 0x1.4f9b2769d2ca7p+0, 0x1.5342b569d4f82p+0, 0x1.56f4736b527dap+0,
    0x1.5ab07dd485429p+0, 0x1.5e76f15ad2148p+0, 0x1.6247eb03a5585p+0, 0x1.6623882552225p+0,
    0x1.6a09e667f3bcdp+0, 0x1.6dfb23c651a2fp+0, 0x1.71f75e8ec5f74p+0, 0x1.75feb564267c9p+0,
    0x1.7a11473eb0187p+0, 0x1.7e2f336cf4e62p+0, 0x1.82589994cce13p+0, 0x1.868d99b4492edp+0,
    0x1.8ace5422aa0dbp+0, 0x1.8f1ae99157736p+0, 0x1.93737b0cdc5e5p+0, 0x1.97d829fde4e50p+0,
    0x1.9c49182a3f090p+0, 0x1.a0c667b5de565p+0, 0x1.a5503b23e255dp+0, 0x1.a9e6b5579fdbfp+0,
    0x1.ae89f995ad3adp+0, 0x1.b33a2b84f15fbp+0, 0x1.b7f76f2fb5e47p+0, 0x1.bcc1e904bc1d2p+0,
    0x1.c199bdd85529cp+0, 0x1.c67f12e57d14bp+0, 0x1.cb720dcef9069p+0, 0x1.d072d4a07897cp+0,
    0x1.d5818dcfba487p+0, 0x1.da9e603db3285p+0, 0x1.dfc97337b9b5fp+0, 0x1.e502ee78b3ff6p+0,
    0x1.ea4afa2a490dap+0, 0x1.efa1bee615a27p+0, 0x1.f50765b6e4540p+0, 0x1.fa7c1819e90d8p+0,
};
// (cb: called right after the table read is issued — the deferred j side's atomics, n3_step_defer)
struct NoCb {
    __device__ __forceinline__ void operator()() const {}
};
template <typename CB = NoCb>
__device__ __forceinline__ double exp2_neg_cut_tab(double t64, bool keep, const double* tab, CB cb = {}) {
    const double m = __builtin_rint(t64);
    const double g = t64 - m;
    const int mi = (int)m;
    const double te = tab[mi & 63];
    cb();
    double p = 0x1.5d87fe78a6731p-40;
    p = fma(p, g, 0x1.3b2ab6fba4e77p-31);
    p = fma(p, g, 0x1.c6b08d704a0c0p-23);
    p = fma(p, g, 0x1.ebfbdff82c58fp-15);
    p = fma(p, g, 0x1.62e42fefa39efp-7);
    p = fma(p, g, 1.0);
    return ldexp(p * te, keep ? (mi >> 6) : -1100);
}
// the mid tier's 2^t (Newton-3 blocks, pairs >= r_mid apart): the same table times a degree-4 fit of
// 2^(g/64) on g in [-1/2, 1/2] (Chebyshev interpolation in long double, coefficients rounded to double;
// 2.53e-15 relative in double Horner, measured on 200,001 points) — one FMA fewer (kTab4RelErr)
template <typename CB = NoCb>
__device__ __forceinline__ double exp2_neg_cut_tab4(double t64, bool keep, const double* tab, CB cb = {}) {
    const double m = __builtin_rint(t64);
    const double g = t64 - m;
    const int mi = (int)m;
    const double te = tab[mi & 63];
    cb();
    double p = 0x1.3b2ad028fa84ap-31;
    p = fma(p, g, 0x1.c6b0c40d96fd0p-23);
    p = fma(p, g, 0x1.ebfbdff82ac88p-15);
    p = fma(p, g, 0x1.62e42fefa0352p-7);
    p = fma(p, g, 1.0);
    return ldexp(p * te, keep ? (mi >> 6) : -1100);
}
// stage the table (threads 0..63 of the workgroup; before the kernel's first barrier)
__device__ __forceinline__ void stage_exp_tab(double* etab) {
    if (MDQT_EXP_TAB && threadIdx.x < 64) etab[threadIdx.x] = kExp2Tab64[threadIdx.x];
    (void)etab;
}

__device__ __forceinline__ const double* pos_base(const double* Rall, int g, int S) {
    const int w = g / S;
    return Rall + (size_t)w * 3 * S + (g - w * S);
}

// Minimum image dx -= L*round(dx/L) (SpeedUp:218-220), exactly, without the division: for
// |dx/L| < 1.5, round(dx/L) is +1 iff dx >= T and -1 iff dx <= -T, T the smallest double with
// fl(T/L) >= 0.5 (host nextafter search), and dx - copysign(L, dx) is bit-identical to dx - L
// resp. dx + L.  GUARD: positions may have left [-L/8, 9L/8] (set_state input), so take the
// division form for separations beyond G = 1.25 L.
template <bool GUARD>
__device__ __forceinline__ void mic(double& dx, double& dy, double& dz, const PairC& c) {
    if (GUARD && !(fabs(dx) < c.G && fabs(dy) < c.G && fabs(dz) < c.G)) {
        dx -= c.L * round(dx / c.L);
        dy -= c.L * round(dy / c.L);
        dz -= c.L * round(dz / c.L);
        return;
    }
    dx = (fabs(dx) >= c.T) ? dx - copysign(c.L, dx) : dx;
    dy = (fabs(dy) >= c.T) ? dy - copysign(c.L, dy) : dy;
    dz = (fabs(dz) >= c.T) ? dz - copysign(c.L, dz) : dz;
}

// Minimum image of the fast variant: dx -= L rint(dx / L) with the reciprocal (3 operations per
// axis, any |dx|).  It differs from the reference's round(dx/L) only when dx/L lies within an ulp
// of +-1/2, i.e. for pairs on the cutoff shell r ~ L/2 (with the other two separations below
// ~1e-7 L for the pair to fall inside the cutoff either way): a measure-zero event.
__device__ __forceinline__ void mic_r(double& dx, double& dy, double& dz, const PairC& c) {
    dx = fma(-__builtin_rint(dx * c.invL), c.L, dx);
    dy = fma(-__builtin_rint(dy * c.invL), c.L, dy);
    dz = fma(-__builtin_rint(dz * c.invL), c.L, dz);
}

template <int VARIANT, bool GUARD>
__device__ __forceinline__ void mic_v(double& dx, double& dy, double& dz, const PairC& c) {
    if (VARIANT == 1) mic_r(dx, dy, dz, c);
    else mic<GUARD>(dx, dy, dz, c);
}

// Force factor ft of one minimum-image separation (F_i += d * ft), 0 unless 0 < r < L/2
// (:221-224).  Branch-free: out-of-range values are discarded by the final select.
template <int VARIANT>
__device__ __forceinline__ double pair_ft(double dx, double dy, double dz, const PairC& c) {
    if (VARIANT == 0) {
        const double r2 = dx * dx + dy * dy + dz * dz;
        const double dr = sqrt(r2);
        const double ft = (1. / dr + c.invlDeb) * exp(-dr / c.lDeb) / (dr * dr);   // :224
        return (dr > 0 && dr < c.Rcut) ? ft : 0.;
    } else {
        const double r2 = fma(dx, dx, fma(dy, dy, dz * dz));
        const double ri = rsq3(r2);
        const double dr = r2 * ri;
        const double ft = ((ri + c.invlDeb) * exp2_neg(dr * (c.invlDeb * kNegLog2e))) * (ri * ri);
        if (VARIANT == 2)                        // the reference's pair set: r2 as :216, exact cutoff
            return (dx * dx + dy * dy + dz * dz < c.rc2 && r2 > 0) ? ft : 0.;
        return (dr < c.Rcut) ? ft : 0.;          // r2 = 0 (coincident ions) gives dr = NaN: 0
    }
}

// Pair potential exp(-r/lDeb)/r (:265), 0 unless 0 < r < L/2
template <int VARIANT>
__device__ __forceinline__ double pair_u(double dx, double dy, double dz, const PairC& c) {
    if (VARIANT == 0) {
        const double dr = sqrt(dx * dx + dy * dy + dz * dz);
        const double u = exp(-dr / c.lDeb) / (dr);
        return (dr > 0 && dr < c.Rcut) ? u : 0.;
    } else {
        const double r2 = fma(dx, dx, fma(dy, dy, dz * dz));
        const double ri = rsq3(r2);
        const double dr = r2 * ri;
        const double u = exp2_neg(dr * (c.invlDeb * kNegLog2e)) * ri;
        return (dr < c.Rcut) ? u : 0.;           // r2 = 0 gives dr = NaN: 0
    }
}

// The fast variant for the Newton-3 tile kernels (no self pairs; pad ions at distinct points):
// pair_ft<1> with the cutoff folded into the 2^t exponent shift (exp2_neg_cut: one 32-bit select
// instead of a 64-bit select of the result; r = 0 must not occur).  Same values as pair_ft<1>.
template <typename CB = NoCb>
__device__ __forceinline__ double pair_ft_cut(double dx, double dy, double dz, const PairC& c, CB cb = {}) {
    const double r2 = fma(dx, dx, fma(dy, dy, dz * dz));
    const double ri = rsq3(r2);
    const double dr = r2 * ri;
    if constexpr (MDQT_EXP_TAB)
        return ((ri + c.invlDeb) * exp2_neg_cut_tab(dr * (c.invlDeb * (64. * kNegLog2e)), dr < c.Rcut, c.etab, cb)) *
               (ri * ri);
    cb();
    return ((ri + c.invlDeb) * exp2_neg_cut(dr * (c.invlDeb * kNegLog2e), dr < c.Rcut)) * (ri * ri);
}

// pair_ft_cut of a mid-range sub-tile group (Newton-3 blocks, gap >= r_mid; MDQT_EXP_TAB): rsq1 and
// the table's 2^t with the degree-4 series — a term within (r/lDeb + 3)(kRsq1RelErr + 2^-52) +
// kTab4RelErr of itself; the cutoff on the f64 r^2 (rsq1's r carries 2e-14: pairs at L/2 would flip)
template <typename CB = NoCb>
__device__ __forceinline__ double pair_ft_cut_mid(double dx, double dy, double dz, const PairC& c, CB cb = {}) {
    const double r2 = fma(dx, dx, fma(dy, dy, dz * dz));
    const double ri = rsq1(r2);
    const double dr = r2 * ri;
    return ((ri + c.invlDeb) * exp2_neg_cut_tab4(dr * (c.invlDeb * (64. * kNegLog2e)), r2 < c.rc2, c.etab, cb)) *
           (ri * ri);
}

// pair_ft_cut of a far tile pair (Newton-3 blocks): rsq1 and the degree-6 2^f, within kFarRelErr
__device__ __forceinline__ double pair_ft_cut_far(double dx, double dy, double dz, const PairC& c) {
    const double r2 = fma(dx, dx, fma(dy, dy, dz * dz));
    const double ri = rsq1(r2);
    const double dr = r2 * ri;
    return ((ri + c.invlDeb) * exp2_neg_cut6(dr * (c.invlDeb * kNegLog2e), dr < c.Rcut)) * (ri * ri);
}

// pair_ft_cut of a very far tile pair: the raw v_rsq_f64 and the degree-5 2^f (mdqt_internal.hpp);
// the cutoff on r^2 (c.rc2 = Rcut^2), not on the raw rsq's r (2^-23: pairs at L/2 would flip)
__device__ __forceinline__ double pair_ft_cut_vfar(double dx, double dy, double dz, const PairC& c) {
    const double r2 = fma(dx, dx, fma(dy, dy, dz * dz));
#if defined(__HIP_DEVICE_COMPILE__)
    const double ri = __builtin_amdgcn_rsq(r2);
#else
    const double ri = 1. / sqrt(r2);
#endif
    const double dr = r2 * ri;
    return ((ri + c.invlDeb) * exp2_neg_cut5(dr * (c.invlDeb * kNegLog2e), r2 < c.rc2)) * (ri * ri);
}

// pair_ft_cut of an ultra-far tile pair: the raw v_rsq_f64 and 2^t by v_exp_f32 (t rounded to
// float; the cutoff as t = -inf, whose 2^t is +0)
__device__ __forceinline__ double pair_ft_cut_ufar(double dx, double dy, double dz, const PairC& c) {
    const double r2 = fma(dx, dx, fma(dy, dy, dz * dz));
#if defined(__HIP_DEVICE_COMPILE__)
    const double ri = __builtin_amdgcn_rsq(r2);
#else
    const double ri = 1. / sqrt(r2);
#endif
    const double dr = r2 * ri;
    const float tf = r2 < c.rc2 ? (float)(dr * (c.invlDeb * kNegLog2e)) : -INFINITY;   // (as vfar)
#if defined(__HIP_DEVICE_COMPILE__)
    const double e = (double)__builtin_amdgcn_exp2f(tf);
#else
    const double e = (double)exp2f(tf);
#endif
    return ((ri + c.invlDeb) * e) * (ri * ri);
}

// The pair potential u = e^(-r/lDeb) / r (SpeedUp:265) in the error-bounded forms of the Newton-3
// blocks (Epotential() on the plan, round 6): level FAR's rsq and 2^t, the same cutoff, u = 2^t ri.  A
// term's relative error is at most the force form's err(r) (one factor ri instead of three), and
// u(r) = g(r) r lDeb / (r + lDeb) < lDeb g(r), so every ion's U_i is within lDeb x (the force tiers'
// per-ion bound) of its exact-form sum (mdqt_engine.cpp potential_rows)
template <int FAR>
__device__ __forceinline__ double pair_u_cut(double dx, double dy, double dz, const PairC& c) {
    static_assert(FAR >= 1 && FAR <= 4, "the exact form is pair_u");
    const double r2 = fma(dx, dx, fma(dy, dy, dz * dz));
    if constexpr (FAR == 1 || FAR == 2) {
        const double ri = rsq1(r2);
        const double dr = r2 * ri;
        if constexpr (FAR == 1)
            return exp2_neg_cut_tab4(dr * (c.invlDeb * (64. * kNegLog2e)), r2 < c.rc2, c.etab) * ri;
        return exp2_neg_cut6(dr * (c.invlDeb * kNegLog2e), dr < c.Rcut) * ri;
    } else {
#if defined(__HIP_DEVICE_COMPILE__)
        const double ri = __builtin_amdgcn_rsq(r2);
#else
        const double ri = 1. / sqrt(r2);
#endif
        const double dr = r2 * ri;
        if constexpr (FAR == 3) return exp2_neg_cut5(dr * (c.invlDeb * kNegLog2e), r2 < c.rc2) * ri;
        const float tf = r2 < c.rc2 ? (float)(dr * (c.invlDeb * kNegLog2e)) : -INFINITY;
#if defined(__HIP_DEVICE_COMPILE__)
        return (double)__builtin_amdgcn_exp2f(tf) * ri;
#else
        return (double)exp2f(tf) * ri;
#endif
    }
}

template <int VARIANT>
__device__ __forceinline__ void accum(double& f, double d, double ft) {
    if (VARIANT == 0) f += d * ft;        // the reference's F[i] += dx*ftotal (:225-230)
    else f = fma(d, ft, f);
}

// ------------------------------------------------------------------------------------------
// Newton-3 tile pairs: one workgroup (4 waves) per tile pair (I, J), I <= J.  Lane l holds ion
// I*64 + l; the J tile sits in LDS twice over (positions j and j + 64), so at rotation step s
// lane l meets ion J*64 + ((l + s) & 63) at LDS index l + s (an immediate offset in the unrolled
// loop).  Each distinct pair is evaluated once: +f goes to the i accumulator (registers), +f to
// the j accumulator (ds_add_f64 at index l + s; the wave's LDS operations run in order, so the
// accumulation order is fixed), and the j side is negated at the end (exact).  Wave q takes
// rotation steps [16q, 16q + 16) (diagonal tile: lane distances 1 + 8q .. 8 + 8q, the 32nd only
// for lanes < 32).  The four waves' partials are combined in a fixed order and written to slot
// J (rows of I) and slot I (rows of J); the diagonal tile's two sides are summed into slot I.
// F = canonical sum of the ntiles slots (seg_sum).  Deterministic, no global atomics.
// ------------------------------------------------------------------------------------------
// one rotation step of a Newton-3 tile pair: lane's ion i against the J-tile ion at LDS index
// idx; +f to the i accumulator (registers) and to the j accumulator (ds_add_f64, no return)
// SHIFT (fast variant, spatial order): every pair of the tile pair has the same minimum-image
// multiples n (one per axis), and the caller passes the i position already shifted, xi - n L
// (MDQT_SHIFT_I; n = 0 on most axes, where it is the same value), so no per-pair image operation;
// with MDQT_SHIFT_I 0 the multiples nsh are applied per pair, bit for bit mic_r's fma.
#ifndef MDQT_SHIFT_I
#define MDQT_SHIFT_I 1
#endif
// POT: Epotential's pair potential u (pair_u) instead of the force: u to the i accumulator fx and
// to the j accumulator ax only (both sides of a pair get +u)
// the pair terms of one rotation step: the lane's i ion against the J-tile ion at LDS index idx —
// the force components (px, py, pz) to the i accumulator; returns them for the j side (POT: u in px)
// MAX >= 0 (Newton-3 blocks, a tile pair whose image varies on one axis only): the caller passes the
// i position shifted on the other two axes (as SHIFT), and the minimum image is taken per pair on axis
// MAX alone — mic_r's operations on that axis, none on the others
// J positions in LDS: the arrays pj[3][128] (generic pointer), or (MDQT_LDS_SPLIT) one LDS address per
// component, made opaque at every rotation step by the caller — so that the compiler cannot merge two
// steps' reads into one ds_read2_b64 (8 LDS cycles per wave for 2 x 512 B, where two ds_read_b64 take 2 + 2;
// MI355X_MICROARCH.md §LDS) nor needs a v_add_u32 for a base beyond read2's 8-bit offset field
#ifndef MDQT_LDS_SPLIT
#define MDQT_LDS_SPLIT 0
#endif
typedef __attribute__((address_space(3))) const double* lds_dp;
struct LdsPJ { lds_dp x, y, z; };
__device__ __forceinline__ double pj_at(const double (*pj)[128], int c, int idx) { return pj[c][idx]; }
__device__ __forceinline__ double pj_at(const LdsPJ& p, int c, int idx) { return (c == 0 ? p.x : c == 1 ? p.y : p.z)[idx]; }
__device__ __forceinline__ LdsPJ lds_pj(const double (*pj)[128], int b) {   // component bases at index b
    return LdsPJ{(lds_dp)&pj[0][b], (lds_dp)&pj[1][b], (lds_dp)&pj[2][b]};
}
__device__ __forceinline__ void lds_pj_opaque(LdsPJ& p) { asm volatile("" : "+v"(p.x), "+v"(p.y), "+v"(p.z)); }

// SC (the tile kernel's box-scaled form, MDQT_N3_SCALED): xi and the J tile hold x / L (rounded once at
// load: a position perturbation within 1 ulp of the box, ~2.7e-15 at C2 — the positions' own storage
// rounding); the minimum image ds - rint(ds) (2 operations per axis instead of 3), r_s = r / L, and the
// force of the physical pair from ds: F = ds (ri_s / L^2 + 1 / (lDeb L)) e^(-r/lDeb) ri_s^2 — the same
// operation count as the unscaled form, 3 VALU fewer per pair
template <int VARIANT, bool GUARD, bool RAGGED, bool SHIFT = false, bool CUT = false, bool POT = false,
          int FAR = 0, int MAX = -1, typename PJ = const double (*)[128], bool SC = false, typename CB = NoCb>
__device__ __forceinline__ void n3_terms(int idx, double m, double xi, double yi, double zi, double mi,
                                         PJ pj, const double* mj, double& fx, double& fy,
                                         double& fz, const PairC& c, const double* nsh, double& px, double& py,
                                         double& pz, CB cb = {}) {
    // cb (n3_step_defer): after this step's LDS reads are issued — the 2^t table's read in the forms that
    // have one, the J positions' otherwise
    constexpr bool TAB = MDQT_EXP_TAB && !POT && (SC || FAR == 1 || (FAR == 0 && CUT));
    double dx = xi - pj_at(pj, 0, idx), dy = yi - pj_at(pj, 1, idx), dz = zi - pj_at(pj, 2, idx);   // :213-215
    if constexpr (!TAB) cb();
    if constexpr (SC) {
        static_assert(VARIANT == 1 && CUT && !POT && !FAR && MAX < 0 && !SHIFT && MDQT_EXP_TAB, "the scaled tile form");
        dx -= __builtin_rint(dx);                   // minimum image in box units (SpeedUp:218-220)
        dy -= __builtin_rint(dy);
        dz -= __builtin_rint(dz);
        const double r2 = fma(dx, dx, fma(dy, dy, dz * dz));
        const double ri = rsq3(r2);
        const double dr = r2 * ri;                  // r / L; the cutoff r < L/2 as r / L < 1/2
        double ft = (fma(ri, c.sA, c.sB) * exp2_neg_cut_tab(dr * c.sT, dr < 0.5, c.etab, cb)) * (ri * ri);
        if (RAGGED) ft *= mi * mj[idx];
        ft *= m;
        px = dx * ft; py = dy * ft; pz = dz * ft;
        fx += px; fy += py; fz += pz;
        return;
    }
    if constexpr (SHIFT) {
        if (!MDQT_SHIFT_I) {
            dx = fma(-nsh[0], c.L, dx);             // = mic_r's fma(-rint(dx / L), L, dx)
            dy = fma(-nsh[1], c.L, dy);
            dz = fma(-nsh[2], c.L, dz);
        }
    } else if constexpr (MAX >= 0) {
        static_assert(VARIANT == 1 && MDQT_SHIFT_I && MAX < 3, "one-axis image: the fast variant, i shifted");
        double& d = MAX == 0 ? dx : MAX == 1 ? dy : dz;
        d = fma(-__builtin_rint(d * c.invL), c.L, d);
    } else {
        mic_v<VARIANT, GUARD>(dx, dy, dz, c);
    }
    if constexpr (POT) {
        // FAR > 0: the error-bounded forms of a Newton-3 block plan (pair_u_cut); 0: the exact form
        double u;
        if constexpr (FAR > 0) u = pair_u_cut<FAR>(dx, dy, dz, c);
        else u = pair_u<VARIANT>(dx, dy, dz, c);
        if (RAGGED) u *= mi * mj[idx];
        u *= m;
        fx += u;
        px = u; py = 0.; pz = 0.;
        (void)fy; (void)fz;
        return;
    }
    static_assert(!FAR || CUT, "the far pair forms are the fast variant's");
    static_assert(FAR != 1 || MDQT_EXP_TAB, "the mid tier's 2^t is the table's");
    // FAR: 0 exact form, 1 mid, 2 far, 3 very far, 4 ultra far (Newton-3 blocks, error-bounded)
    double ft = FAR == 4 ? pair_ft_cut_ufar(dx, dy, dz, c)
              : FAR == 3 ? pair_ft_cut_vfar(dx, dy, dz, c)
              : FAR == 2 ? pair_ft_cut_far(dx, dy, dz, c)
              : FAR == 1 ? pair_ft_cut_mid(dx, dy, dz, c, cb)
              : CUT ? pair_ft_cut(dx, dy, dz, c, cb) : pair_ft<VARIANT>(dx, dy, dz, c);
    if (RAGGED) ft *= mi * mj[idx];
    ft *= m;
    px = dx * ft; py = dy * ft; pz = dz * ft;
    fx += px; fy += py; fz += pz;
}

// one rotation step: the pair terms, +f to the i accumulator (registers) and to the j accumulator
// (ds_add_f64 at index idx, no return; one wave's LDS operations run in order, so the
// accumulation order is fixed)
template <int VARIANT, bool GUARD, bool RAGGED, bool SHIFT = false, bool CUT = false, bool POT = false,
          int FAR = 0, int MAX = -1, typename PJ = const double (*)[128], bool SC = false>
__device__ __forceinline__ void n3_step(int idx, double m, double xi, double yi, double zi, double mi,
                                        PJ pj, const double* mj, double* ax, double* ay,
                                        double* az, double& fx, double& fy, double& fz, const PairC& c,
                                        const double* nsh = nullptr) {
    double px, py, pz;
    n3_terms<VARIANT, GUARD, RAGGED, SHIFT, CUT, POT, FAR, MAX, PJ, SC>(idx, m, xi, yi, zi, mi, pj, mj, fx, fy, fz, c, nsh, px,
                                                                py, pz);
#if defined(MDQT_EXPT_NOJACC)
    (void)ax; (void)ay; (void)az;
#else
    __hip_atomic_fetch_add(&ax[idx], px, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    if constexpr (!POT) {
        __hip_atomic_fetch_add(&ay[idx], py, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __hip_atomic_fetch_add(&az[idx], pz, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
#endif
}

// the j-side atomics of one step (n3_step's, split out for the deferred form)
template <bool POT>
__device__ __forceinline__ void n3_j_add(int idx, double* ax, double* ay, double* az, double px, double py, double pz) {
#if defined(MDQT_EXPT_NOJACC)
    (void)idx; (void)ax; (void)ay; (void)az; (void)px; (void)py; (void)pz;
#else
    __hip_atomic_fetch_add(&ax[idx], px, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    if constexpr (!POT) {
        __hip_atomic_fetch_add(&ay[idx], py, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __hip_atomic_fetch_add(&az[idx], pz, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
    }
#endif
}
// MDQT_N3_DEFER_J: one rotation step with its j side one step late — the pair terms of step idx, then the
// previous step's j terms (q*, at index qidx >= 0) to LDS, and this step's kept in q* for the next.  A
// wave's LDS operations complete in order, so the next step's position and table reads wait behind the
// atomics issued before them; deferred, those atomics are a step older.  The same adds in the same order
// per accumulator entry: bit for bit n3_step.
#ifndef MDQT_N3_DEFER_J
#define MDQT_N3_DEFER_J 0
#endif
template <int VARIANT, bool GUARD, bool RAGGED, bool SHIFT = false, bool CUT = false, bool POT = false,
          int FAR = 0, int MAX = -1, typename PJ = const double (*)[128], bool SC = false>
__device__ __forceinline__ void n3_step_defer(int idx, double m, double xi, double yi, double zi, double mi,
                                              PJ pj, const double* mj, double* ax, double* ay,
                                              double* az, double& fx, double& fy, double& fz, const PairC& c,
                                              const double* nsh, int qidx, double& qx, double& qy, double& qz) {
    double px, py, pz;
    auto prev = [&]() {
        if (qidx >= 0) n3_j_add<POT>(qidx, ax, ay, az, qx, qy, qz);
    };
    n3_terms<VARIANT, GUARD, RAGGED, SHIFT, CUT, POT, FAR, MAX, PJ, SC>(idx, m, xi, yi, zi, mi, pj, mj, fx, fy, fz, c, nsh,
                                                                       px, py, pz, prev);
    qx = px; qy = py; qz = pz;
}

#ifndef MDQT_N3_WAVES
#define MDQT_N3_WAVES 4
#endif
constexpr int N3W = MDQT_N3_WAVES;                  // waves per tile pair (2, 4 or 8)
static_assert(N3W == 2 || N3W == 4 || N3W == 8, "waves per tile pair");

// the j accumulators of the N3W waves, both halves of each, combined in wave order
__device__ __forceinline__ double n3_jsum(const double (*accj)[3][128], int k, int l) {
    double w = accj[0][k][l] + accj[0][k][l + 64];
#pragma unroll
    for (int q = 1; q < N3W; ++q) w += accj[q][k][l] + accj[q][k][l + 64];
    return w;
}

// slot stores: plain, or write-through (sc1) when the QT launch of an overlapped MD step reads
// them after an arrival count instead of a kernel boundary (MI355X_MICROARCH.md, hand-off forms)
#ifndef MDQT_EXPT_SIGMODE
#define MDQT_EXPT_SIGMODE 0     // diagnostic builds: 1 = no arrival atomics, 2 = plain slot stores
#endif
// Every tile-pair slot store is write-through (agent scope): the slots stream out while the
// kernel runs instead of sitting dirty in the XCDs' L2s for the kernel-end write-back that makes
// them visible to the QT launch's waves on other XCDs.  A/B at C2: force launch 16.8 -> 16.2 us,
// MD step -0.6 us.  0: plain stores (A/B builds).
#ifndef MDQT_SLOT_WT
#define MDQT_SLOT_WT 1
#endif
template <bool SIG>
__device__ __forceinline__ void slot_store(double* p, double v) {
    if constexpr (MDQT_EXPT_SIGMODE != 2 && (SIG || MDQT_SLOT_WT))   // SIGMODE 2: plain stores
        __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}

#ifndef MDQT_N3_CUT
#define MDQT_N3_CUT 1
#endif
#ifndef MDQT_N3_SCALED
#define MDQT_N3_SCALED 1                            // the tile kernel's box-scaled force form (n3_terms SC); A/B round 6: C2 force launch -4 %
#endif
#ifndef MDQT_N3_PRIO
#define MDQT_N3_PRIO 0
#endif
template <int VARIANT, bool GUARD, bool RAGGED, bool SIG, bool POT = false>
__device__ __forceinline__ void n3_tile(const N3Args& a, const PairC& c, int I, int J,
                                        double (*pj)[128], double (*accj)[3][128], double* mj,
                                        double (*ia)[3][64]) {
    constexpr bool CUT = VARIANT == 1 && MDQT_N3_CUT;   // pair_ft_cut
    // a part of the tile pair (the split table, mdqt_engine.cpp tile_split_count): I's bits 30-31 = log2 of
    // the parts (0 whole, 1 halves, 2 quarters), bits 28-29 = which part — each wave's rotation steps in
    // that many consecutive runs; part p > 0 writes its rows into the extra slot ntiles + p - 1 (a diagonal
    // tile's second half: ntiles + 3)
    const int pl = (int)((unsigned)I >> 30), part = (I >> 28) & 3;
    I &= 0x0FFFFFFF;
    static_assert(N3W == 4, "the split table assumes 16 rotation steps per wave");
    const int q = threadIdx.x >> 6, l = threadIdx.x & 63;
    const int S = a.S, N = a.N;
    const double* X = a.R;
    const double* Y = a.R + S;
    const double* Z = a.R + 2 * S;
    // the box-scaled force form (MDQT_N3_SCALED): positions in box units from the load on
    constexpr bool SC = MDQT_N3_SCALED && VARIANT == 1 && CUT && !POT && !GUARD && MDQT_EXP_TAB;
    const double sc = SC ? c.invL : 1.;
    PairC cs = c;
    if constexpr (SC) {
        cs.sA = c.invL * c.invL;
        cs.sB = c.invlDeb * c.invL;
        cs.sT = c.L * (c.invlDeb * (64. * kNegLog2e));
    }
    if (q == 0) {                                   // stage the J tile (twice over)
        const int j = J * 64 + l;
        const bool vj = !RAGGED || j < N;
        // pad ions (ragged last tile): distinct points (pad-pad pairs must have r > 0), weight 0
        const double pad = (double)(l + 1) * 0x1p-10;
        double xj = vj ? X[j] : pad, yj = vj ? Y[j] : pad, zj = vj ? Z[j] : pad;
        if constexpr (SC) { xj *= sc; yj *= sc; zj *= sc; }
        pj[0][l] = xj; pj[0][l + 64] = xj;
        pj[1][l] = yj; pj[1][l + 64] = yj;
        pj[2][l] = zj; pj[2][l + 64] = zj;
        if (RAGGED) { mj[l] = vj ? 1. : 0.; mj[l + 64] = mj[l]; }
    }
#pragma unroll
    for (int k = 0; k < 3; ++k) { accj[q][k][l] = 0.; accj[q][k][l + 64] = 0.; }
    const int i = I * 64 + l;
    const bool vi = !RAGGED || i < N;
    const double padi = (double)(l + 1) * 0x1p-10;
    double xi = vi ? X[i] : padi, yi = vi ? Y[i] : padi, zi = vi ? Z[i] : padi;
    if constexpr (SC) { xi *= sc; yi *= sc; zi *= sc; }
    const double mi = vi ? 1. : 0.;
    __syncthreads();
    double fx = 0., fy = 0., fz = 0.;
    double* ax = accj[q][0];
    double* ay = accj[q][1];
    double* az = accj[q][2];
    LdsPJ pb{};                                     // MDQT_LDS_SPLIT: the bases at the loop's first index
    int pbase = 0;
    auto set_base = [&](int b) {
        if constexpr (MDQT_LDS_SPLIT) { pb = lds_pj(pj, b); pbase = b; }
    };
    double qx = 0., qy = 0., qz = 0.;              // MDQT_N3_DEFER_J: the previous step's j terms, at qidx
    int qidx = -1;
    auto step = [&](int idx, double m) {
        if constexpr (MDQT_N3_DEFER_J) {
            n3_step_defer<VARIANT, GUARD, RAGGED, false, CUT, POT, 0, -1, const double (*)[128], SC>(
                idx, m, xi, yi, zi, mi, pj, mj, ax, ay, az, fx, fy, fz, cs, nullptr, qidx, qx, qy, qz);
            qidx = idx;
        } else if constexpr (MDQT_LDS_SPLIT) {      // (the LDS bases opaque per step: ds_read_b64, no read2)
            lds_pj_opaque(pb);
            n3_step<VARIANT, GUARD, RAGGED, false, CUT, POT, 0, -1, LdsPJ, SC>(idx - pbase, m, xi, yi, zi, mi, pb,
                                                                              mj + pbase, ax + pbase, ay + pbase,
                                                                              az + pbase, fx, fy, fz, cs);
        } else {
            n3_step<VARIANT, GUARD, RAGGED, false, CUT, POT, 0, -1, const double (*)[128], SC>(
                idx, m, xi, yi, zi, mi, pj, mj, ax, ay, az, fx, fy, fz, cs);
        }
    };
    const bool diag = I == J;
    // progress priority (MDQT_N3_PRIO): a SIMD's VALU issue goes to the highest-priority wave, then
    // the oldest, so without it the oldest of a SIMD's 6-7 co-resident waves run ahead and the last
    // ones finish alone, latency-bound (stamps: workgroup end times rise with the dispatch order).
    // Each wave lowers its priority as it advances through its steps (3, 2, 1, 0 per quarter): the
    // waves behind are issued first, the co-resident waves progress together and the SIMD stays
    // full to the end.
    auto prio = [&](int t, int n) {
        if constexpr (MDQT_N3_PRIO) {
            if (t == 0) __builtin_amdgcn_s_setprio(3);         // (immediate operands: t is a
            else if (t == n / 4) __builtin_amdgcn_s_setprio(2);   // constant of the unrolled loop)
            else if (t == n / 2) __builtin_amdgcn_s_setprio(1);
            else if (t == 3 * n / 4) __builtin_amdgcn_s_setprio(0);
        }
    };
    if (!diag && pl) {                              // steps [part 16 / 2^pl, (part + 1) 16 / 2^pl)
        const int b = l + (64 / N3W) * q + part * ((64 / N3W) >> pl);
        set_base(b);
        if (pl == 1) {
#pragma unroll
            for (int t = 0; t < 8; ++t) step(b + t, 1.);
        } else {
#pragma unroll
            for (int t = 0; t < 4; ++t) step(b + t, 1.);
        }
    } else if (diag && pl) {                        // a diagonal tile's 8 steps per wave in two halves
        const int b = l + 1 + (32 / N3W) * q + 4 * part;
        set_base(b);
#pragma unroll
        for (int t = 0; t < 3; ++t) step(b + t, 1.);
        step(b + 3, (part == 1 && q == N3W - 1 && l >= 32) ? 0. : 1.);   // lane distance 32: once per pair
    } else if (!diag) {
        const int b = l + (64 / N3W) * q;
        set_base(b);
#pragma unroll
        for (int t = 0; t < 64 / N3W; ++t) {
            prio(t, 64 / N3W);
            step(b + t, 1.);
        }
    } else {
        const int b = l + 1 + (32 / N3W) * q;
        set_base(b);
#pragma unroll
        for (int t = 0; t < 32 / N3W - 1; ++t) {
            prio(t, 32 / N3W);
            step(b + t, 1.);
        }
        step(b + 32 / N3W - 1, (q == N3W - 1 && l >= 32) ? 0. : 1.);  // lane distance 32: once per pair
    }
    if constexpr (MDQT_N3_PRIO) __builtin_amdgcn_s_setprio(0);
    if constexpr (MDQT_N3_DEFER_J) {
        if (qidx >= 0) n3_j_add<POT>(qidx, ax, ay, az, qx, qy, qz);
    }
    ia[q][0][l] = fx; ia[q][1][l] = fy; ia[q][2][l] = fz;
    __syncthreads();
    const size_t slab3 = POT ? (size_t)S : (size_t)3 * S;   // potential: [ntiles][S], one plane per slot
    constexpr int NK = POT ? 1 : 3;                 // potential: component 0 only, j side not negated
    const int xs = part == 0 ? -1 : diag ? a.ntiles + 3 : a.ntiles + part - 1;   // a later part's extra slot
    if (q == 0) {                                   // rows of I -> slot J (diagonal: I; a later part: xs)
        double* Pi = a.P + (size_t)(xs >= 0 ? xs : J) * slab3;
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            double v = ia[0][k][l];
#pragma unroll
            for (int w = 1; w < N3W; ++w) v += ia[w][k][l];
            if (diag) v = POT ? v + n3_jsum(accj, k, l) : v - n3_jsum(accj, k, l);
            if (i < S) slot_store<SIG>(&Pi[(size_t)k * S + i], v);
        }
    } else if (q == 1 && !diag) {                   // rows of J -> slot I (a later part: xs)
        double* Pj = a.P + (size_t)(xs >= 0 ? xs : I) * slab3;
        const int j = J * 64 + l;
#pragma unroll
        for (int k = 0; k < NK; ++k) {
            const double w = n3_jsum(accj, k, l);
            if (j < S) slot_store<SIG>(&Pj[(size_t)k * S + j], POT ? w : -w);
        }
    }
    if constexpr (SIG) {                            // every storing wave drained, then one arrival
        // Release/acquire hand-off (the consumer polls with acquire, mdqt_qtfast.hip): the
        // workgroup's slot stores happen-before its barrier, the barrier before thread 0's
        // agent-scope release, so a consumer that acquires the count sees them.  On gfx950 the
        // release is an L2 write-back — the price of these options (off by default, §8).
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (MDQT_EXPT_SIGMODE != 1 && threadIdx.x == 0) {   // one arrival per tile whose rows were written
            __hip_atomic_fetch_add(a.arrive + I, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
            if (J != I) __hip_atomic_fetch_add(a.arrive + J, 1ull, __ATOMIC_RELEASE, __HIP_MEMORY_SCOPE_AGENT);
        }
    }
}

}  // namespace mdqt
