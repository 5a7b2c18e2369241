// Device helpers shared by the gfx950 QT kernels (mdqt_kernels.hip, mdqt_qtfast.hip):
// Philox stream, complex helpers, the QT arithmetic modes, sincos, DPP/LDS lane moves.
#pragma once

#include "mdqt_internal.hpp"

#include <math.h>

namespace mdqt {

// ------------------------------------------------------------------------------------------
// Philox4x32-10 (Salmon et al. SC'11): the counter-based stream keyed by (seed, job) with
// counter (global ion, qstep index, draw pair); layout in DESIGN.md §RNG (the parity tests
// check it against the CPU restatement's stream).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ void philox4x32_10(uint32_t c0, uint32_t c1, uint32_t c2, uint32_t c3,
                                              uint32_t k0, uint32_t k1, uint32_t o[4]) {
#pragma unroll
    for (int r = 0; r < 10; ++r) {
        const uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        const uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        const uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        const uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        const uint32_t n0 = hi1 ^ c1 ^ k0, n2 = hi0 ^ c3 ^ k1;
        c0 = n0; c1 = lo1; c2 = n2; c3 = lo0;
        k0 += 0x9E3779B9u; k1 += 0xBB67AE85u;
    }
    o[0] = c0; o[1] = c1; o[2] = c2; o[3] = c3;
}

__device__ __forceinline__ double u53(uint32_t hi, uint32_t lo) {
    const uint64_t b = ((((uint64_t)hi) << 32) | lo) >> 11;
    return (double)b * 0x1.0p-53;
}

// draws 2p and 2p+1 of (ion, q)
__device__ __forceinline__ void philox_pair(const QTConst& qc, uint64_t ion, uint64_t q, int p,
                                            double& ua, double& ub) {
    uint32_t o[4];
    philox4x32_10((uint32_t)ion, (uint32_t)q, (uint32_t)(q >> 32),
                  ((uint32_t)(ion >> 32) << 8) | (uint32_t)p, qc.seed, qc.job, o);
    ua = u53(o[0], o[1]);
    ub = u53(o[2], o[3]);
}

// uniforms 2p, 2p+1 of local ion i at substep (gid, q): the precomputed drand48 reference-order
// values when U is given (rng_mode 0), else the Philox stream
__device__ __forceinline__ void draw_pair(const QTConst& qc, const double* U, int S, int i, uint64_t gid,
                                          uint64_t q, int p, double& ua, double& ub) {
    if (U) {
        ua = U[(size_t)(2 * p) * S + i];
        ub = (2 * p + 1 < 5) ? U[(size_t)(2 * p + 1) * S + i] : 0.;
    } else {
        philox_pair(qc, gid, q, p, ua, ub);
    }
}

struct cxd { double re, im; };

__device__ __forceinline__ cxd cmul(cxd a, cxd b) {   // std::complex<double> operator*
    return {a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re};
}
__device__ __forceinline__ cxd cadd(cxd a, cxd b) { return {a.re + b.re, a.im + b.im}; }

// The two QT arithmetic modes (option "qt_math"): F = false keeps the reference's operations
// without contraction (bit-identical to the oracle up to sin/cos ulps); F = true contracts into
// FMAs and takes 1/sqrt(1 - dp) from a refined v_rsq_f64 (a few ulp per operation).
template <bool F>
__device__ __forceinline__ cxd cmulT(cxd a, cxd b) {
    if (F) return {fma(a.re, b.re, -(a.im * b.im)), fma(a.re, b.im, a.im * b.re)};
    return cmul(a, b);
}
template <bool F>
__device__ __forceinline__ double decay_term(cxd y, double d) {   // (re d) re + (im d) im
    if (F) return fma(y.re * d, y.re, (y.im * d) * y.im);
    return (y.re * d) * y.re + (y.im * d) * y.im;
}
template <bool F>
__device__ __forceinline__ double inv_sqrt_1m(double dp) {        // 1 / sqrt(1 - dp) (:532)
    if (F) {
        const double x = 1 - dp;
        double r = __builtin_amdgcn_rsq(x);
        const double hx = 0.5 * x;
        r = r * fma(-hx * r, r, 1.5);
        r = r * fma(-hx * r, r, 1.5);
        return r;
    }
    return 1 / sqrt(1 - dp);
}
template <bool F>
__device__ __forceinline__ double axpy(double a, double x, double y) {   // y + a x
    if (F) return fma(a, x, y);
    return y + a * x;
}
template <bool F>
__device__ __forceinline__ double kstage(double invh, double pref, double ws, double y) {
    if (F) return invh * fma(pref, ws, -y);                         // invh (pref ws - y)
    return invh * (pref * ws - y);
}

// 1 / sqrt(x) (F) or the reference's division by sqrt(x): the renormalisation of :706-712
template <bool F>
__device__ __forceinline__ cxd renorm_div(cxd w, double sumsq) {
    if (F) {
        double r = __builtin_amdgcn_rsq(sumsq);
        const double hx = 0.5 * sumsq;
        r = r * fma(-hx * r, r, 1.5);
        r = r * fma(-hx * r, r, 1.5);
        return {w.re * r, w.im * r};
    }
    const double nrm = sqrt(sumsq);
    return {w.re / nrm, w.im / nrm};
}

// sin and cos of the time-dependent coupling phase (:508).  F = false: the math library's
// sincos.  F = true: Cody-Waite reduction by pi/2 (three-part constant, FMA) and the classic
// minimax kernels on [-pi/4, pi/4] (fdlibm's __kernel_sin/__kernel_cos coefficients, < 1 ulp),
// about a third of the library's instruction count; |x| >= 2^20 takes the library path.
#ifndef MDQT_FAST_SINCOS
#define MDQT_FAST_SINCOS 1
#endif
// Horner step z * p + c as one three-address v_fma_f64.  (With the coefficient c held in a VGPR —
// the lane kernel's SGPRs are all taken — the compiler otherwise emits a copy of c and the
// two-address v_fmac_f64: one extra VALU per step.)  Same operation, same value as fma(z, p, c).
__device__ __forceinline__ double hfma(double z, double p, double c) {
#if defined(__HIP_DEVICE_COMPILE__)
    double r;
    asm("v_fma_f64 %0, %1, %2, %3" : "=v"(r) : "v"(z), "v"(p), "v"(c));
    return r;
#else
    return fma(z, p, c);
#endif
}
// the reduction + kernels without the range check (valid for |x| < 2^20), branch-free
__device__ __forceinline__ void sincos_fast(double x, double& sn, double& cs) {
    const double n = rint(x * 0.63661977236758134308);           // 2/pi
    double r = fma(-n, 1.57079632679489655800e+00, x);            // pi/2 = P1 + P2 + P3
    r = fma(-n, 6.12323399573676603587e-17, r);
    r = fma(-n, -1.49738490485916983014e-33, r);
    const double z = r * r;
    const double ps = hfma(z, hfma(z, hfma(z, hfma(z, 1.58969099521155010221e-10, -2.50507602534068634195e-08),
                                           2.75573137070700676789e-06), -1.98412698298579493134e-04),
                           8.33333333332248946124e-03);
    const double sr = fma(r * z, hfma(z, ps, -1.66666666666666324348e-01), r);
    const double pc = z * hfma(z, hfma(z, hfma(z, hfma(z, hfma(z, -1.13596475577881948265e-11, 2.08757232129817482790e-09),
                                                    -2.75573143513906633035e-07), 2.48015872894767294178e-05),
                                   -1.38888888888741095749e-03), 4.16666666666666019037e-02);
    const double hz = 0.5 * z;
    const double wc = 1.0 - hz;
    const double cr = wc + (((1.0 - wc) - hz) + z * pc);
    const int q = (int)n & 3;
    const double s0 = (q & 1) ? cr : sr, c0 = (q & 1) ? sr : cr;
    sn = (q & 2) ? -s0 : s0;
    cs = ((q + 1) & 2) ? -c0 : c0;
}
template <bool F>
__device__ __forceinline__ void sincos_q(double x, double& sn, double& cs) {
    if (!F || !MDQT_FAST_SINCOS || !(fabs(x) < 1048576.)) {
        sincos(x, &sn, &cs);
        return;
    }
    sincos_fast(x, sn, cs);
}

// e^(ix) through a 64-entry table (the qt_math 2 kernels' coupling phase, round 3): x = m (2 pi/64)
// + r by the same FMA Cody-Waite reduction (three-part constant), |r| <= pi/64, then
// e^(ix) = e^(2 pi i (m mod 64)/64) e^(ir) with e^(ir) by its Taylor series (sin to r^9, cos to
// r^8: truncation below 1e-20) and the table entries correctly rounded (60-digit decimal
// arithmetic).  22 VALU and one LDS read instead of sincos_fast's ~40; <= 2 ulp.  |x| < 2^20 (the
// callers take the library beyond).  `tab`: kSinCos64 (cos, sin pairs) in LDS or global memory.
#ifndef MDQT_QT_SCTAB
#define MDQT_QT_SCTAB 1
#endif
static __constant__ const double kSinCos64[128] = {
    0x1.0000000000000p+0, 0x0.0p+0, 0x1.fd88da3d12526p-1, 0x1.917a6bc29b42cp-4,
    0x1.f6297cff75cb0p-1, 0x1.8f8b83c69a60bp-3, 0x1.e9f4156c62ddap-1, 0x1.294062ed59f06p-2,
    0x1.d906bcf328d46p-1, 0x1.87de2a6aea963p-2, 0x1.c38b2f180bdb1p-1, 0x1.e2b5d3806f63bp-2,
    0x1.a9b66290ea1a3p-1, 0x1.1c73b39ae68c8p-1, 0x1.8bc806b151741p-1, 0x1.44cf325091dd6p-1,
    0x1.6a09e667f3bcdp-1, 0x1.6a09e667f3bcdp-1, 0x1.44cf325091dd6p-1, 0x1.8bc806b151741p-1,
    0x1.1c73b39ae68c8p-1, 0x1.a9b66290ea1a3p-1, 0x1.e2b5d3806f63bp-2, 0x1.c38b2f180bdb1p-1,
    0x1.87de2a6aea963p-2, 0x1.d906bcf328d46p-1, 0x1.294062ed59f06p-2, 0x1.e9f4156c62ddap-1,
    0x1.8f8b83c69a60bp-3, 0x1.f6297cff75cb0p-1, 0x1.917a6bc29b42cp-4, 0x1.fd88da3d12526p-1,
    0x1.84054757668f0p-192, 0x1.0000000000000p+0, -0x1.917a6bc29b42cp-4, 0x1.fd88da3d12526p-1,
    -0x1.8f8b83c69a60bp-3, 0x1.f6297cff75cb0p-1, -0x1.294062ed59f06p-2, 0x1.e9f4156c62ddap-1,
    -0x1.87de2a6aea963p-2, 0x1.d906bcf328d46p-1, -0x1.e2b5d3806f63bp-2, 0x1.c38b2f180bdb1p-1,
    -0x1.1c73b39ae68c8p-1, 0x1.a9b66290ea1a3p-1, -0x1.44cf325091dd6p-1, 0x1.8bc806b151741p-1,
    -0x1.6a09e667f3bcdp-1, 0x1.6a09e667f3bcdp-1, -0x1.8bc806b151741p-1, 0x1.44cf325091dd6p-1,
    -0x1.a9b66290ea1a3p-1, 0x1.1c73b39ae68c8p-1, -0x1.c38b2f180bdb1p-1, 0x1.e2b5d3806f63bp-2,
    -0x1.d906bcf328d46p-1, 0x1.87de2a6aea963p-2, -0x1.e9f4156c62ddap-1, 0x1.294062ed59f06p-2,
    -0x1.f6297cff75cb0p-1, 0x1.8f8b83c69a60bp-3, -0x1.fd88da3d12526p-1, 0x1.917a6bc29b42cp-4,
    -0x1.0000000000000p+0, 0x1.7e0478355de7fp-191, -0x1.fd88da3d12526p-1, -0x1.917a6bc29b42cp-4,
    -0x1.f6297cff75cb0p-1, -0x1.8f8b83c69a60bp-3, -0x1.e9f4156c62ddap-1, -0x1.294062ed59f06p-2,
    -0x1.d906bcf328d46p-1, -0x1.87de2a6aea963p-2, -0x1.c38b2f180bdb1p-1, -0x1.e2b5d3806f63bp-2,
    -0x1.a9b66290ea1a3p-1, -0x1.1c73b39ae68c8p-1, -0x1.8bc806b151741p-1, -0x1.44cf325091dd6p-1,
    -0x1.6a09e667f3bcdp-1, -0x1.6a09e667f3bcdp-1, -0x1.44cf325091dd6p-1, -0x1.8bc806b151741p-1,
    -0x1.1c73b39ae68c8p-1, -0x1.a9b66290ea1a3p-1, -0x1.e2b5d3806f63bp-2, -0x1.c38b2f180bdb1p-1,
    -0x1.87de2a6aea963p-2, -0x1.d906bcf328d46p-1, -0x1.294062ed59f06p-2, -0x1.e9f4156c62ddap-1,
    -0x1.8f8b83c69a60bp-3, -0x1.f6297cff75cb0p-1, -0x1.917a6bc29b42cp-4, -0x1.fd88da3d12526p-1,
    -0x1.2a033eb3aa9dbp-190, -0x1.0000000000000p+0, 0x1.917a6bc29b42cp-4, -0x1.fd88da3d12526p-1,
    0x1.8f8b83c69a60bp-3, -0x1.f6297cff75cb0p-1, 0x1.294062ed59f06p-2, -0x1.e9f4156c62ddap-1,
    0x1.87de2a6aea963p-2, -0x1.d906bcf328d46p-1, 0x1.e2b5d3806f63bp-2, -0x1.c38b2f180bdb1p-1,
    0x1.1c73b39ae68c8p-1, -0x1.a9b66290ea1a3p-1, 0x1.44cf325091dd6p-1, -0x1.8bc806b151741p-1,
    0x1.6a09e667f3bcdp-1, -0x1.6a09e667f3bcdp-1, 0x1.8bc806b151741p-1, -0x1.44cf325091dd6p-1,
    0x1.a9b66290ea1a3p-1, -0x1.1c73b39ae68c8p-1, 0x1.c38b2f180bdb1p-1, -0x1.e2b5d3806f63bp-2,
    0x1.d906bcf328d46p-1, -0x1.87de2a6aea963p-2, 0x1.e9f4156c62ddap-1, -0x1.294062ed59f06p-2,
    0x1.f6297cff75cb0p-1, -0x1.8f8b83c69a60bp-3, 0x1.fd88da3d12526p-1, -0x1.917a6bc29b42cp-4,
};
__device__ __forceinline__ void sincos_tab(double x, const double* tab, double& sn, double& cs) {
    const double m = __builtin_rint(x * 0x1.45f306dc9c883p+3);      // 64 / (2 pi)
    double r = fma(-m, 0x1.921fb54442d18p-4, x);                      // 2 pi / 64 = C1 + C2 + C3
    r = fma(-m, 0x1.1a62633145c07p-58, r);
    r = fma(-m, -0x1.f1976b7ed8fbcp-114, r);
    const int j = (int)m & 63;
    const double tc = tab[2 * j], ts = tab[2 * j + 1];
    const double z = r * r;
    const double sr = fma(r * z, hfma(z, hfma(z, hfma(z, 2.7557319223985893e-06, -1.9841269841269841e-04),
                                               8.3333333333333332e-03), -1.6666666666666666e-01), r);
    const double cr = hfma(z, hfma(z, hfma(z, hfma(z, 2.4801587301587302e-05, -1.3888888888888889e-03),
                                         4.1666666666666664e-02), -0.5), 1.0);
    sn = fma(ts, cr, tc * sr);
    cs = fma(tc, cr, -(ts * sr));
}
// the qt_math 2 kernels' phase: the table form (MDQT_QT_SCTAB) or sincos_fast, the library for
// |x| >= 2^20
__device__ __forceinline__ void sincos_q2(double x, const double* tab, double& sn, double& cs) {
    if (!(fabs(x) < 1048576.)) {
        sincos(x, &sn, &cs);
        return;
    }
    if (MDQT_QT_SCTAB) sincos_tab(x, tab, sn, cs);
    else sincos_fast(x, sn, cs);
}

__device__ __forceinline__ double rho_im(cxd a, cxd b) {   // Im(a * conj(b)), SpeedUp:490-502
    return a.re * (-b.im) + a.im * b.re;
}

__device__ __forceinline__ double gat(double v, int src) {
    const int lo = __builtin_amdgcn_ds_bpermute(src << 2, __double2loint(v));
    const int hi = __builtin_amdgcn_ds_bpermute(src << 2, __double2hiint(v));
    return __hiloint2double(hi, lo);
}
__device__ __forceinline__ cxd gatc(cxd v, int src) { return {gat(v.re, src), gat(v.im, src)}; }

// DPP moves inside a 16-lane row (one ion): row_shl:n (lane l reads lane l+n), row_shr:n
// (lane l reads lane l-n), row_newbcast:n (every lane reads lane n of its row).  VALU-latency
// cross-lane moves for the fixed-pattern sums; exact.
// Row gathers of the sparse matvec through LDS (one ds_write_b128 + three ds_read_b128 per
// exchange) instead of twelve ds_bpermute_b32; the 16-lane group lives in one wave, whose LDS
// operations execute in order, so a wave-scope fence is the only synchronisation needed.
#ifndef MDQT_GATHER_LDS
#define MDQT_GATHER_LDS 1
#endif
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

template <int CTRL>
__device__ __forceinline__ double dpp(double v) {
    // row_newbcast is a DP-ALU DPP control on gfx950: one v_mov_b64_dpp moves the whole double
    if constexpr (CTRL >= 0x150 && CTRL <= 0x15F) return __builtin_amdgcn_update_dpp(0., v, CTRL, 0xF, 0xF, true);
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, true);
    return __hiloint2double(hi, lo);
}
#define SHL(n) (0x100 + (n))
#define SHR(n) (0x110 + (n))
#define BCAST(n) (0x150 + (n))
#define ROR(n) (0x120 + (n))
#define QP_XOR1 0xB1   // quad_perm [1, 0, 3, 2]: lane ^ 1
#define QP_XOR2 0x4E   // quad_perm [2, 3, 0, 1]: lane ^ 2

// ((T2 + T3) + T4) + T5 of the ion's lanes 2..5, in every lane of the row
__device__ __forceinline__ double row_sum_p(double T) {
    double a = T + dpp<SHL(1)>(T);
    a = a + dpp<SHL(2)>(T);
    a = a + dpp<SHL(3)>(T);
    return dpp<BCAST(2)>(a);
}


}  // namespace mdqt
