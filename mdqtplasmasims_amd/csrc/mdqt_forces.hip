// gfx950 force kernels: forces() (SpeedUp:192-236) and the pair potential of Epotential()
// (SpeedUp:244-281).
//
//   k_pairs<MODE, VARIANT>   owner-computes rows, LDS-staged j tiles, j split in segments
//   k_pairs_n3<VARIANT>      Newton-3 over 64x64 tile pairs, 4 waves per pair (one GPU)
//   k_reduce_segments        canonical sum of the partials when a caller asks for F
//
// VARIANT 0 keeps the reference's operations (sqrt, the three divisions, libm exp) without
// contraction; VARIANT 1 (default) is the reciprocal form (rsq3) with a range-specialised exp and
// FMA contraction — a few ulp per pair, inside the 1e-13 force gate.  VARIANT 2 (Newton-3
// tiles; the MC + MD program, whose lattice start puts pairs exactly on the cutoff and on the
// image boundary) has variant 1's values with variant 0's pair set: the exact minimum image and
// the cutoff as r2 < rc2, rc2 the smallest double with sqrt(rc2) >= Rcut.
#include "mdqt_internal.hpp"
#include "mdqt_pairs.hpp"

#include <math.h>

namespace mdqt {

// ------------------------------------------------------------------------------------------
// rows: owner computes row i over the j of its segment in ASCENDING j (the single-thread
// reference's F_i is exactly that sum; the self pair has r = 0 and is dropped
// by the 0 < r test like the reference's coincident pairs)
// ------------------------------------------------------------------------------------------
constexpr int FT = 256;

template <int MODE, int VARIANT, bool GUARD>
__device__ __forceinline__ void rows_body(const ForceArgs& a, const PairC& c, double* sx, double* sy,
                                          double* sz) {
    const int tid = threadIdx.x;
    const int li = blockIdx.x * FT + tid;
    const int seg = blockIdx.y;
    const bool active = li < a.nrows;
    const int gi = a.row_lo + li;
    double rx = 0., ry = 0., rz = 0.;
    if (active) {
        const double* p = pos_base(a.Rall, gi, a.S);
        rx = p[0]; ry = p[a.S]; rz = p[2 * a.S];
    }
    double fx = 0., fy = 0., fz = 0.;
    const int j0 = seg * a.seglen;
    const int j1 = min(a.N, j0 + a.seglen);
    for (int jt = j0; jt < j1; jt += FT) {
        const int jl = jt + tid;
        __syncthreads();
        if (jl < j1) {
            const double* p = pos_base(a.Rall, jl, a.S);
            sx[tid] = p[0]; sy[tid] = p[a.S]; sz[tid] = p[2 * a.S];
        }
        __syncthreads();
        const int nj = min(FT, j1 - jt);
        if (active) {
#pragma unroll 2
            for (int k = 0; k < nj; ++k) {
                double dx = rx - sx[k], dy = ry - sy[k], dz = rz - sz[k];   // :213-215
                mic_v<VARIANT, GUARD>(dx, dy, dz, c);
                if (MODE == 0) {
                    const double ft = pair_ft<VARIANT>(dx, dy, dz, c);
                    accum<VARIANT>(fx, dx, ft);
                    accum<VARIANT>(fy, dy, ft);
                    accum<VARIANT>(fz, dz, ft);
                } else {
                    const double u = pair_u<VARIANT>(dx, dy, dz, c);
                    if (VARIANT == 0) fx += u;
                    else fx += u;
                }
            }
        }
    }
    if (active) {
        double* o = a.Fpart + (size_t)seg * 3 * a.S;
        o[li] = fx;
        if (MODE == 0) { o[a.S + li] = fy; o[2 * a.S + li] = fz; }
    }
}

template <int MODE, int VARIANT, bool GUARD>
__global__ __launch_bounds__(FT) void k_pairs(ForceArgs a) {
    __shared__ double sx[FT], sy[FT], sz[FT];
    const PairC c = {a.L, a.micT, a.micGuard, a.Rcut, a.lDeb, a.invlDeb, 1. / a.L};
    rows_body<MODE, VARIANT, GUARD>(a, c, sx, sy, sz);
}

__global__ __launch_bounds__(256) void k_reduce_segments(const double* __restrict__ Fpart,
                                                         double* __restrict__ F, int nseg,
                                                         int nrows, int S, int ncomp, size_t plane) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    const int c = blockIdx.y;
    if (i >= nrows || c >= ncomp) return;
    F[(size_t)c * S + i] = slot_sum16(Fpart + (size_t)c * S + i, plane, nseg);
}

#if defined(MDQT_EXPT_STAMPS)
// diagnostic build only: per-workgroup start/end (s_memrealtime, 100 MHz) and placement
__device__ unsigned long long g_n3_stamps[6 * 8192];
#endif

template <int VARIANT, bool GUARD>
__global__ __launch_bounds__(64 * N3W) void k_pairs_n3(N3Args a) {
    __shared__ double pj[3][128];
    __shared__ double accj[N3W][3][128];
    __shared__ double ia[N3W][3][64];
    __shared__ double mj[128];
    __shared__ double etab[64];
#if defined(MDQT_EXPT_STAMPS)
    const unsigned long long t_start = __builtin_amdgcn_s_memrealtime();
    const unsigned long long c_start = __builtin_amdgcn_s_memtime();
#endif
    stage_exp_tab(etab);
    const int2 IJ = a.pairs[blockIdx.x];
    const PairC c = {a.L, a.micT, a.micGuard, a.Rcut, a.lDeb, a.invlDeb, 1. / a.L, a.rc2, etab};
    const bool rag = (a.N & 63) && IJ.y == a.ntiles - 1;
    if (a.arrive) {
        if (rag) n3_tile<VARIANT, GUARD, true, true>(a, c, IJ.x, IJ.y, pj, accj, mj, ia);
        else n3_tile<VARIANT, GUARD, false, true>(a, c, IJ.x, IJ.y, pj, accj, mj, ia);
    } else {
        if (rag) n3_tile<VARIANT, GUARD, true, false>(a, c, IJ.x, IJ.y, pj, accj, mj, ia);
        else n3_tile<VARIANT, GUARD, false, false>(a, c, IJ.x, IJ.y, pj, accj, mj, ia);
    }
#if defined(MDQT_EXPT_STAMPS)
    __syncthreads();
    if (threadIdx.x == 0 && blockIdx.x < 8192) {
        const unsigned long long t_end = __builtin_amdgcn_s_memrealtime();
        const unsigned long long c_end = __builtin_amdgcn_s_memtime();
        g_n3_stamps[6 * blockIdx.x] = t_start;
        g_n3_stamps[6 * blockIdx.x + 1] = t_end;
        g_n3_stamps[6 * blockIdx.x + 2] = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_ID
        g_n3_stamps[6 * blockIdx.x + 3] = __builtin_amdgcn_s_getreg((31 << 11) | 20);   // XCC_ID
        g_n3_stamps[6 * blockIdx.x + 4] = c_start;                                       // core clock
        g_n3_stamps[6 * blockIdx.x + 5] = c_end;
    }
#endif
}

// Epotential() (:244-281) on the Newton-3 tiles: each distinct pair's u once, to both ions' rows
// (slot component 0; the caller sums the ntiles slots per ion)
template <int VARIANT, bool GUARD>
__global__ __launch_bounds__(64 * N3W) void k_pairs_n3_pot(N3Args a) {
    __shared__ double pj[3][128];
    __shared__ double accj[N3W][3][128];
    __shared__ double ia[N3W][3][64];
    __shared__ double mj[128];
    const int2 IJ = a.pairs[blockIdx.x];
    const PairC c = {a.L, a.micT, a.micGuard, a.Rcut, a.lDeb, a.invlDeb, 1. / a.L, a.rc2};
    const bool rag = (a.N & 63) && IJ.y == a.ntiles - 1;
    if (rag) n3_tile<VARIANT, GUARD, true, false, true>(a, c, IJ.x, IJ.y, pj, accj, mj, ia);
    else n3_tile<VARIANT, GUARD, false, false, true>(a, c, IJ.x, IJ.y, pj, accj, mj, ia);
}

#if defined(MDQT_EXPT_STAMPS)
extern "C" int mdqt_expt_n3_stamps(unsigned long long* out, int n) {
    return hipMemcpyFromSymbol(out, HIP_SYMBOL(g_n3_stamps), sizeof(unsigned long long) * 6 * n) == hipSuccess ? 0 : -1;
}
#endif

// ------------------------------------------------------------------------------------------
// Newton-3 over BLOCK pairs (large N, one GPU or sharded): blocks of 16 tiles (1024 ions); a
// workgroup of 16 waves holds block P (wave q: tile I = 16P + q in registers) and walks the
// block distances db of its run, db in [0, NB/2] of the cyclic half shell (block Q = P + db mod
// NB; db = NB/2 only from P < NB/2 when NB is even; db = 0: tile pairs I <= J).  For every J
// tile of Q all 16 waves run their (I, J) rotation (64 steps; 32 on the diagonal tile) against
// the J tile in LDS with per-wave j accumulators, which are then combined in wave order and
// written to j-slot db (rows of J); each wave's i accumulator spans the whole run and goes to
// i-slot nd + run.  Slots: [nd + R][3][Npad], nd = NB/2 + 1 — O(N^2/1024) doubles, not O(N^2/64).
// The canonical per-ion sum (k_n3b_reduce) takes the j-slots in db order, then the i-slots in
// run order, skipping slots this rank does not write.
// ------------------------------------------------------------------------------------------
constexpr int BW = 16;                              // tiles per block = waves per workgroup
#if defined(MDQT_EXPT_CLS)
// diagnostic build only: tile-pair classes of k_pairs_n3b (skip, per pair, uniform image)
__device__ unsigned long long g_cls_count[3];
extern "C" int mdqt_expt_cls_count(unsigned long long* out, int reset) {
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_cls_count), sizeof(unsigned long long) * 3) != hipSuccess) return -1;
    if (reset) {
        const unsigned long long z[3] = {0, 0, 0};
        if (hipMemcpyToSymbol(HIP_SYMBOL(g_cls_count), z, sizeof(z)) != hipSuccess) return -1;
    }
    return 0;
}
#endif

__device__ __forceinline__ double uniform_f64(double v) {   // a wave-uniform value into SGPRs
    return __hiloint2double(__builtin_amdgcn_readfirstlane(__double2hiint(v)),
                            __builtin_amdgcn_readfirstlane(__double2loint(v)));
}

__device__ __forceinline__ const double* tile_base(const double* Rall, int tile, int S) {
    const int g = tile * 64;                        // S is a multiple of 64: tiles never straddle slabs
    const int w = g / S;
    return Rall + (size_t)w * 3 * S + (g - w * S);
}

// steps whose j-side terms are combined in registers before one LDS atomic (block kernel; 1 = every
// step its own ds_add_f64)
#ifndef MDQT_N3B_JCOMB
#define MDQT_N3B_JCOMB 1
#endif
constexpr int kJComb = MDQT_N3B_JCOMB;
static_assert(kJComb == 1 || kJComb == 2 || kJComb == 4 || kJComb == 8 || kJComb == 16, "j-side step groups");
__device__ __forceinline__ double wave_rol1(double v) {   // lane l <- lane (l + 1) mod 64
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), 0x134, 0xF, 0xF, false);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), 0x134, 0xF, 0xF, false);
    return __hiloint2double(hi, lo);
}

template <int VARIANT, bool GUARD, bool RAGGED, bool SHIFT = false, bool CUT = VARIANT == 1 && MDQT_N3_CUT,
          bool POT = false, int FAR = 0>
__device__ __forceinline__ void n3b_pair(bool diag, int l, double xi, double yi, double zi, double mi,
                                         const double (*pj)[128], const double* mj, double* ax, double* ay,
                                         double* az, double& fx, double& fy, double& fz, const PairC& c,
                                         const double* nsh = nullptr) {
    // every 16 steps the LDS arrays are re-based at the lane's index (an opaque register), so the
    // 16 unrolled steps address them with immediate offsets t, 128 + t, 256 + t: without it the
    // compiler's strength reduction moved the base past the arrays and spent a v_add_u32 per
    // ds_add_f64 (3.5 VALU per pair, ~8 % of the block kernel's instructions)
#define N3B_REBASE(b0)                                                                     \
    int b_ = (b0);                                                                         \
    asm volatile("" : "+v"(b_));                                                           \
    const double (*pjb)[128] = (const double (*)[128])(&pj[0][0] + b_);                    \
    const double* mjb = mj + b_;                                                           \
    double *axb = ax + b_, *ayb = ay + b_, *azb = az + b_
    if constexpr (kJComb > 1) {
        // j side combined over kJComb consecutive steps before one ds_add_f64 per component: at
        // step t lane l's pair is with J index l + t, at step t + 1 lane l + 1's is too, so the
        // running sum rotated one lane down (wave_rol:1, lane l reads lane l + 1) plus this step's
        // term is the sum for lane l's current J index; lane 63 receives lane 0's sum, whose index
        // differs by 64 — the same J ion (the tile sits in LDS twice, the halves summed at the end)
        auto group = [&](auto&& pjb, const double* mjb, double* axb, double* ayb, double* azb, int t, double m,
                         double& jx, double& jy, double& jz) {
            double px, py, pz;
            n3_terms<VARIANT, GUARD, RAGGED, SHIFT, CUT, POT, FAR>(t, m, xi, yi, zi, mi, pjb, mjb, fx, fy, fz, c, nsh,
                                                                   px, py, pz);
            if (t % kJComb == 0) {
                jx = px; jy = py; jz = pz;
            } else {
                jx = wave_rol1(jx) + px;
                if constexpr (!POT) { jy = wave_rol1(jy) + py; jz = wave_rol1(jz) + pz; }
            }
            if (t % kJComb == kJComb - 1) {
                __hip_atomic_fetch_add(&axb[t], jx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                if constexpr (!POT) {
                    __hip_atomic_fetch_add(&ayb[t], jy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                    __hip_atomic_fetch_add(&azb[t], jz, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
                }
            }
        };
        if (!diag) {
            for (int t0 = 0; t0 < 64; t0 += 16) {
                N3B_REBASE(l + t0);
                double jx = 0., jy = 0., jz = 0.;
#pragma unroll
                for (int t = 0; t < 16; ++t) group(pjb, mjb, axb, ayb, azb, t, 1., jx, jy, jz);
            }
        } else {
            for (int t0 = 1; t0 < 33; t0 += 16) {
                N3B_REBASE(l + t0);
                double jx = 0., jy = 0., jz = 0.;
#pragma unroll
                for (int t = 0; t < 16; ++t)
                    group(pjb, mjb, axb, ayb, azb, t, (t0 + t == 32 && l >= 32) ? 0. : 1., jx, jy, jz);
            }
        }
    } else if (!diag) {
        for (int t0 = 0; t0 < 64; t0 += 16) {
            N3B_REBASE(l + t0);
#pragma unroll
            for (int t = 0; t < 16; ++t)
                n3_step<VARIANT, GUARD, RAGGED, SHIFT, CUT, POT, FAR>(t, 1., xi, yi, zi, mi, pjb, mjb, axb, ayb, azb,
                                                                      fx, fy, fz, c, nsh);
        }
    } else {
        for (int t0 = 1; t0 < 33; t0 += 16) {
            N3B_REBASE(l + t0);
#pragma unroll
            for (int t = 0; t < 16; ++t) {
                const double m = (t0 + t == 32 && l >= 32) ? 0. : 1.;   // lane distance 32: once
                n3_step<VARIANT, GUARD, RAGGED, SHIFT, CUT, POT, FAR>(t, m, xi, yi, zi, mi, pjb, mjb, axb, ayb, azb,
                                                                      fx, fy, fz, c, nsh);
            }
        }
    }
#undef N3B_REBASE
}

#ifndef MDQT_UFAR32_PK
#define MDQT_UFAR32_PK 0   // packed f32 (v_pk_*): measured slower at N = 1M (329.6-330.5 vs 325.6-327.2 ms, A/B)
#endif
__device__ __forceinline__ float wave_rol1f(float v) {   // lane l <- lane (l + 1) mod 64
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x134, 0xF, 0xF, false));
}

// An ultra-far tile pair (boxes >= r_ufar32 apart) with a uniform image, pair terms in f32
// (MDQT_UFAR32; error analysis and bound in mdqt_internal.hpp kUfar32A/B): dx = fl32(xi - n L - xj)
// from the f64 separation, v_rsq_f32, 2^t by v_exp_f32, the cutoff on the f32 r^2 (t = -inf).  Per 16-step group the i side is summed in f32 registers and then added to the
// f64 partial, and the j side runs as MDQT_N3B_JCOMB does (the running sum rotated one lane down
// each step, wave_rol:1 folded into the f32 add: lane l + 1's sum of the previous step has lane l's
// current J index) and ends in one ds_add_f64 per component at the group's last index.  Off the
// diagonal only (a tile's pair with itself is never ultra far).
// (its separations take xi already shifted by n L: there is no per-pair image form of it)
static_assert(MDQT_SHIFT_I || !MDQT_UFAR32, "the f32 ultra-far form needs MDQT_SHIFT_I");
__device__ __forceinline__ void n3b_pair_uf32(int l, double xi, double yi, double zi, const double (*pj)[128],
                                              double* ax, double* ay, double* az, double& fx, double& fy,
                                              double& fz, float cf, float invlf, float rc2f) {
    for (int t0 = 0; t0 < 64; t0 += 16) {
        int b_ = l + t0;
        asm volatile("" : "+v"(b_));                // immediate LDS offsets (N3B_REBASE)
        const double (*pjb)[128] = (const double (*)[128])(&pj[0][0] + b_);
        float ix = 0.f, iy = 0.f, iz = 0.f, jx = 0.f, jy = 0.f, jz = 0.f;
#if MDQT_UFAR32_PK
        // two steps per iteration in packed f32 (v_pk_mul/add/fma_f32: two lanes' worth per
        // instruction); the i side in two interleaved sums, combined at the group's end
        typedef float f2 __attribute__((ext_vector_type(2)));
        f2 ix2 = {0.f, 0.f}, iy2 = {0.f, 0.f}, iz2 = {0.f, 0.f};
        const f2 cf2 = {cf, cf}, il2 = {invlf, invlf};
#pragma unroll
        for (int t = 0; t < 16; t += 2) {
            const f2 dx = {(float)(xi - pjb[0][t]), (float)(xi - pjb[0][t + 1])};
            const f2 dy = {(float)(yi - pjb[1][t]), (float)(yi - pjb[1][t + 1])};
            const f2 dz = {(float)(zi - pjb[2][t]), (float)(zi - pjb[2][t + 1])};
            const f2 r2 = __builtin_elementwise_fma(dx, dx, __builtin_elementwise_fma(dy, dy, dz * dz));
            const f2 ri = {__builtin_amdgcn_rsqf(r2.x), __builtin_amdgcn_rsqf(r2.y)};
            const f2 tt = (r2 * ri) * cf2;
            const f2 e = {__builtin_amdgcn_exp2f(r2.x < rc2f ? tt.x : -INFINITY),
                          __builtin_amdgcn_exp2f(r2.y < rc2f ? tt.y : -INFINITY)};
            const f2 ft = ((ri + il2) * e) * (ri * ri);
            const f2 px = dx * ft, py = dy * ft, pz = dz * ft;
            ix2 += px; iy2 += py; iz2 += pz;
            if (t == 0) {
                jx = px.x; jy = py.x; jz = pz.x;
            } else {
                jx = wave_rol1f(jx) + px.x; jy = wave_rol1f(jy) + py.x; jz = wave_rol1f(jz) + pz.x;
            }
            jx = wave_rol1f(jx) + px.y; jy = wave_rol1f(jy) + py.y; jz = wave_rol1f(jz) + pz.y;
        }
        ix = ix2.x + ix2.y; iy = iy2.x + iy2.y; iz = iz2.x + iz2.y;
#else
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const float dx = (float)(xi - pjb[0][t]), dy = (float)(yi - pjb[1][t]), dz = (float)(zi - pjb[2][t]);
            const float r2 = fmaf(dx, dx, fmaf(dy, dy, dz * dz));
            const float ri = __builtin_amdgcn_rsqf(r2);
            const float e = __builtin_amdgcn_exp2f(r2 < rc2f ? (r2 * ri) * cf : -INFINITY);
            const float ft = ((ri + invlf) * e) * (ri * ri);
            const float px = dx * ft, py = dy * ft, pz = dz * ft;
            if (t == 0) {
                ix = px; iy = py; iz = pz;
                jx = px; jy = py; jz = pz;
            } else {
                ix += px; iy += py; iz += pz;
                jx = wave_rol1f(jx) + px; jy = wave_rol1f(jy) + py; jz = wave_rol1f(jz) + pz;
            }
        }
#endif
        __hip_atomic_fetch_add(ax + b_ + 15, (double)jx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __hip_atomic_fetch_add(ay + b_ + 15, (double)jy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __hip_atomic_fetch_add(az + b_ + 15, (double)jz, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        fx += (double)ix; fy += (double)iy; fz += (double)iz;
    }
}

// POT: Epotential's pair potential (component 0 of the slots, both rows +u) instead of the force
template <int VARIANT, bool GUARD, bool POT = false>
// the fast variant fits 64 VGPRs (8 waves per SIMD); the exact one (libm exp, divisions) gets 128
__global__ __launch_bounds__(BW * 64) __attribute__((amdgpu_waves_per_eu(VARIANT == 1 ? 8 : 4, VARIANT == 1 ? 8 : 4)))
void k_pairs_n3b(N3BArgs a) {
    __shared__ double pj[3][128];
    __shared__ double mj[128];
    __shared__ double accj[BW][3][128];
    __shared__ double irun[BW][3][64];
    __shared__ double etab[64];
    stage_exp_tab(etab);
    const int q = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;   // q: wave-uniform
    const int P = a.Plo + (int)blockIdx.x / a.R;
    const int run = (int)blockIdx.x % a.R;
    const int d0 = run * a.runlen, d1 = min(a.nd, d0 + a.runlen);
    const PairC c = {a.L, a.micT, a.micGuard, a.Rcut, a.lDeb, a.invlDeb, 1. / a.L, a.rc2, etab};
    const int T = a.T, N = a.N, S = a.S;
    const bool ragN = (N & 63) != 0;
    const int I = P * BW + q;
    const bool vI = I < T;
    const int i = I * 64 + l;
    // positions: the sorted copy [3][Npad] (spatial order) or the gathered slabs
    const bool srt = a.use_sort != 0;
    const int PS = srt ? a.Npad : S;
    auto tile_ptr = [&](int tile) { return srt ? a.Rs + tile * 64 : tile_base(a.Rall, tile, S); };
    const double pad = (double)(l + 1) * 0x1p-10;  // pad ions: distinct points (pair_ft_cut: r > 0)
    double xi = pad, yi = pad, zi = pad, mi = 0.;
    if (vI && i < N) {
        const double* p = tile_ptr(I) + l;
        xi = p[0]; yi = p[PS]; zi = p[2 * PS]; mi = 1.;
    }
    // Tile-pair classes in spatial order (SpeedUp:222 keeps a pair only below r = L/2), decided
    // for all BW waves' tile pairs (I, J) by the staging wave's lanes 0..BW-1 into tp[q]:
    //  * skip (force_sort 1): boxes >= L/2 apart in the minimum image — no pair inside the
    //    cutoff, the tile pair adds exact zeros;
    //  * uniform image: every pair's raw separation fl(xi - xj) lies in [fl(lo_I - hi_J),
    //    fl(hi_I - lo_J)] (rounding is monotone), and so does rint(fl(dx / L)) between the rints
    //    of the two ends; equal ends = one minimum-image multiple per axis for every pair, bit for
    //    bit what mic_r computes per pair (the fast variant then skips that rint per pair);
    //  * otherwise the per-pair minimum image.
    // class: -1 skip; otherwise bit 0 = uniform image, + 2 x the far level (1 far pair form, 2 very
    // far, 3 ultra far, 4 ultra far in f32; forces only): 0 .. 9
    __shared__ double tp[BW][4];                    // n_x, n_y, n_z, class
    // skip below the cutoff only for the forces (error-bounded tail, mdqt_engine.cpp tail_radius)
    const double rc2 = POT ? a.Rcut * a.Rcut : a.Rskip * a.Rskip;
    const double rf2 = (POT || VARIANT != 1 || !(a.Rfar < a.Rcut)) ? INFINITY : a.Rfar * a.Rfar;
    const double rv2 = (POT || VARIANT != 1 || !(a.Rvfar < a.Rcut)) ? INFINITY : a.Rvfar * a.Rvfar;
    const double ru2 = (POT || VARIANT != 1 || !(a.Rufar < a.Rcut)) ? INFINITY : a.Rufar * a.Rufar;
    const double ru32 = (POT || VARIANT != 1 || !MDQT_UFAR32 || !(a.Rufar32 < a.Rcut)) ? INFINITY
                                                                                      : a.Rufar32 * a.Rufar32;
    // the f32 form's constants as wave-uniform SGPR values (in VGPRs they were spilled and reloaded
    // inside the pair loop at the kernel's 64-VGPR budget)
    auto sgpr_f = [](float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); };
    const float cf32 = sgpr_f((float)(a.invlDeb * kNegLog2e)), invl32 = sgpr_f((float)a.invlDeb),
                rc2f = sgpr_f((float)a.rc2);
    auto classify = [&](int Iw, int J, double& g2) {   // lane-parallel over Iw (staging wave)
        const double* B = a.boxes;
        g2 = 0.;
        bool uni = true;
        double n[3];
#pragma unroll
        for (int c3 = 0; c3 < 3; ++c3) {
            double d = B[(size_t)c3 * T + Iw] - B[(size_t)c3 * T + J];
            d = fma(-__builtin_rint(d * c.invL), a.L, d);
            const double gap = fabs(d) - (B[(size_t)(3 + c3) * T + Iw] + B[(size_t)(3 + c3) * T + J]);
            g2 = gap > 0. ? fma(gap, gap, g2) : g2;
            const double lo = B[(size_t)(6 + c3) * T + Iw] - B[(size_t)(9 + c3) * T + J];
            const double hi = B[(size_t)(9 + c3) * T + Iw] - B[(size_t)(6 + c3) * T + J];
            const double nlo = __builtin_rint(lo * c.invL), nhi = __builtin_rint(hi * c.invL);
            uni = uni && (nlo == nhi);
            n[c3] = nlo;
        }
        const double cls = (a.use_sort == 1 && g2 > rc2) ? -1.
                                                          : ((VARIANT == 1 && uni) ? 1. : 0.) +
                                                                (g2 > ru32 ? 8. : g2 > ru2 ? 6. : g2 > rv2 ? 4. :
                                                                 g2 > rf2 ? 2. : 0.);
        return make_double4(n[0], n[1], n[2], cls);
    };
    // the run's i accumulator lives in LDS (read and written once per block distance) so that
    // the three-level blocking fits the 64-VGPR budget of two 16-wave workgroups per CU
    double* fi = irun[q][0];
    fi[l] = 0.; fi[64 + l] = 0.; fi[128 + l] = 0.;
    // force_tail_mode 1 (a.tailb): the staging lanes' tail bound of their I tiles (I side, over the
    // whole run) and of the current J tile (J side, summed by thread 0 after the barrier)
    __shared__ double tbi[BW], tbj[BW];
    const bool tmeas = !POT && a.tailb != nullptr;
    if (tmeas && q == 0 && l < BW) tbi[l] = 0.;
    double* ax = accj[q][0];
    double* ay = accj[q][1];
    double* az = accj[q][2];
    const size_t plane = (size_t)3 * a.Npad;
    for (int db = d0; db < d1; ++db) {
        if (!(a.NB & 1) && db == a.NB / 2 && P >= a.NB / 2) continue;   // the other half covers it
        const int Q = (P + db) % a.NB;
        double bx = 0., by = 0., bz = 0.;          // this block distance's i partial (3-level blocking)
        for (int b = 0; b < BW; ++b) {
            const int J = Q * BW + b;
            if (J >= T) break;
            if (q == 0) {                           // stage J (twice over)
                const int j = J * 64 + l;
                const bool vj = j < N;
                const double* p = tile_ptr(J) + l;
                const double xj = vj ? p[0] : pad, yj = vj ? p[PS] : pad, zj = vj ? p[2 * PS] : pad;
                pj[0][l] = xj; pj[0][l + 64] = xj;
                pj[1][l] = yj; pj[1][l + 64] = yj;
                pj[2][l] = zj; pj[2][l + 64] = zj;
                mj[l] = vj ? 1. : 0.; mj[l + 64] = mj[l];
                if (tmeas && l < BW) tbj[l] = 0.;
                if (srt && l < BW && P * BW + l < T) {
                    double g2;
                    const double4 t4 = classify(P * BW + l, J, g2);
                    tp[l][0] = t4.x; tp[l][1] = t4.y; tp[l][2] = t4.z; tp[l][3] = t4.w;
                    // a tile pair skipped by the tail radius (boxes >= Rskip apart) with a pair that
                    // may lie inside L/2: each of its pairs is >= sqrt(g2) apart, so each ion of I
                    // loses at most n_J g(sqrt(g2)) and each ion of J n_I g(sqrt(g2)); counted once per
                    // unordered tile pair (block distance 0: J > I only)
                    const int Iw = P * BW + l;
                    if (tmeas && t4.w < 0. && g2 < a.Rcut * a.Rcut && (db > 0 || J > Iw)) {
                        const double d = sqrt(g2);
                        const double gd = (1. / d + a.invlDeb) * exp(-d / a.lDeb) / d;
                        tbi[l] += (double)min(64, N - J * 64) * gd;
                        tbj[l] = (double)min(64, N - Iw * 64) * gd;
                    }
#if defined(MDQT_EXPT_CLS)
                    atomicAdd(&g_cls_count[t4.w < 0. ? 0 : 1 + ((int)t4.w & 1)], 1ull);
#endif
                }
            }
#pragma unroll
            for (int k = 0; k < 3; ++k) { accj[q][k][l] = 0.; accj[q][k][l + 64] = 0.; }
            __syncthreads();
            if (tmeas && threadIdx.x == 0) {
                double sj = 0.;
                for (int w = 0; w < BW; ++w) sj += tbj[w];
                if (sj > 0.) atomicAdd(a.tailb + J, sj);
            }
            const double cls = srt ? uniform_f64(tp[q][3]) : 0.;
            if (vI && (db > 0 || J >= I) && cls >= 0.) {
                const bool diag = (db == 0 && J == I);
                const int ci = (int)cls;            // bit 0 uniform image, bits 1-3 far level
                const int fl = ci >> 1;
                // blocked i accumulation: the tile pair's 64 steps into a fresh sum, those into the
                // block distance's sum, those into the run's (a run is ~1e5 pair terms at N = 1e6;
                // in spatial order they arrive in coherent groups, and one serial chain would
                // carry their rounding: momentum |sum F| / mean |F| 1.8e-8 -> 1e-10 at C4)
                double tx = 0., ty = 0., tz = 0.;
                constexpr bool CUT = VARIANT == 1 && MDQT_N3_CUT;
                if (ragN && (I == T - 1 || J == T - 1))
                    n3b_pair<VARIANT, GUARD, true, false, CUT, POT>(diag, l, xi, yi, zi, mi, pj, mj, ax, ay, az, tx, ty,
                                                                    tz, c);
                else if (VARIANT == 1 && (ci & 1)) {       // uniform image
                    const double nsh[3] = {uniform_f64(tp[q][0]), uniform_f64(tp[q][1]), uniform_f64(tp[q][2])};
                    // xi - n L once per tile pair (n3_step SHIFT; MDQT_SHIFT_I)
                    const double sx = MDQT_SHIFT_I ? fma(-nsh[0], a.L, xi) : xi;
                    const double sy = MDQT_SHIFT_I ? fma(-nsh[1], a.L, yi) : yi;
                    const double sz = MDQT_SHIFT_I ? fma(-nsh[2], a.L, zi) : zi;
                    if constexpr (VARIANT == 1 && !POT && !GUARD && CUT) {
                        if (fl == 4) {              // ultra far in f32
#if !defined(MDQT_EXPT_UFAR_SKIP)                   // (diagnostic build: skip them, wrong results)
                            n3b_pair_uf32(l, sx, sy, sz, pj, ax, ay, az, tx, ty, tz, cf32, invl32, rc2f);
#endif
                        }
                        else if (fl == 3)           // ultra far tile pair
                            n3b_pair<VARIANT, GUARD, false, true, CUT, POT, 3>(diag, l, sx, sy, sz, mi, pj, mj, ax, ay,
                                                                               az, tx, ty, tz, c, nsh);
                        else if (fl == 2)           // very far tile pair
                            n3b_pair<VARIANT, GUARD, false, true, CUT, POT, 2>(diag, l, sx, sy, sz, mi, pj, mj, ax, ay,
                                                                               az, tx, ty, tz, c, nsh);
                        else if (fl == 1)           // far tile pair: the far pair form
                            n3b_pair<VARIANT, GUARD, false, true, CUT, POT, 1>(diag, l, sx, sy, sz, mi, pj, mj, ax, ay,
                                                                               az, tx, ty, tz, c, nsh);
                        else
                            n3b_pair<VARIANT, GUARD, false, true, CUT, POT>(diag, l, sx, sy, sz, mi, pj, mj, ax, ay,
                                                                            az, tx, ty, tz, c, nsh);
                    } else {
                        n3b_pair<VARIANT, GUARD, false, VARIANT == 1, CUT, POT>(diag, l, sx, sy, sz, mi, pj, mj, ax,
                                                                                ay, az, tx, ty, tz, c, nsh);
                    }
                } else if constexpr (VARIANT == 1 && !POT && !GUARD && CUT) {
                    if (fl >= 2)                    // (ultra far with a per-pair image: rare, very-far form)
                        n3b_pair<VARIANT, GUARD, false, false, CUT, POT, 2>(diag, l, xi, yi, zi, mi, pj, mj, ax, ay,
                                                                            az, tx, ty, tz, c);
                    else if (fl == 1)
                        n3b_pair<VARIANT, GUARD, false, false, CUT, POT, 1>(diag, l, xi, yi, zi, mi, pj, mj, ax, ay,
                                                                            az, tx, ty, tz, c);
                    else
                        n3b_pair<VARIANT, GUARD, false, false, CUT, POT>(diag, l, xi, yi, zi, mi, pj, mj, ax, ay, az,
                                                                         tx, ty, tz, c);
                } else
                    n3b_pair<VARIANT, GUARD, false, false, CUT, POT>(diag, l, xi, yi, zi, mi, pj, mj, ax, ay, az, tx,
                                                                     ty, tz, c);
                bx += tx; by += ty; bz += tz;
            }
            __syncthreads();
            if (q < (POT ? 1 : 3)) {                // j side of J's rows -> j-slot db
                double v = 0.;
#pragma unroll
                for (int w = 0; w < BW; ++w) v = v + (accj[w][q][l] + accj[w][q][l + 64]);
                a.slots[(size_t)db * plane + (size_t)q * a.Npad + J * 64 + l] = POT ? v : -v;
            }
            __syncthreads();
        }
        fi[l] += bx; fi[64 + l] += by; fi[128 + l] += bz;   // one wave's own LDS words: in order
    }
    if (vI) {                                       // i side -> i-slot nd + run
        double* o = a.slots + (size_t)(a.nd + run) * plane + i;
        o[0] = fi[l]; o[a.Npad] = fi[64 + l]; o[2 * (size_t)a.Npad] = fi[128 + l];
    }
    if (tmeas && q == 0 && l < BW && P * BW + l < T && tbi[l] > 0.) atomicAdd(a.tailb + P * BW + l, tbi[l]);
}

// force_tail_mode 1, after the call's per-tile tail sums are complete (all-reduced over the ranks
// when sharded): every tile whose sum, with the sum's rounding (x (1 + 1e-12)), exceeds eps is
// listed for k_tail_fix (this rank's tiles [own_lo, own_hi) only; the count in st[3]); the other
// tiles' largest sum goes into the running maximum st[0] — the bound every ion met after the fix —
// and the largest of all into st[1] (what the skip radius alone gave); st[2] counts every tile
// over eps (the same on every rank: the host widens r_t when it grows), st[4] the measured calls.
// Positive doubles order as their bit patterns.
__global__ __launch_bounds__(256) void k_tail_max(const double* __restrict__ tailb, int T, double eps, int own_lo,
                                                  int own_hi, unsigned long long* st, int* list) {
    double m = 0., mr = 0.;
    unsigned long long nf = 0;
    for (int t = blockIdx.x * 256 + threadIdx.x; t < T; t += gridDim.x * 256) {
        const double v = tailb[t];
        mr = fmax(mr, v);
        if (v * (1. + 1e-12) > eps) {
            ++nf;
            if (t >= own_lo && t < own_hi) list[atomicAdd(st + 3, 1ull)] = t;
        } else {
            m = fmax(m, v);
        }
    }
    for (int off = 32; off > 0; off >>= 1) {
        m = fmax(m, __shfl_xor(m, off));
        mr = fmax(mr, __shfl_xor(mr, off));
        nf += __shfl_xor(nf, off);
    }
    if ((threadIdx.x & 63) == 0) {
        if (m > 0.) atomicMax(st, (unsigned long long)__double_as_longlong(m));
        if (mr > 0.) atomicMax(st + 1, (unsigned long long)__double_as_longlong(mr));
        if (nf) atomicAdd(st + 2, nf);
    }
    if (blockIdx.x == 0 && threadIdx.x == 0) atomicAdd(st + 4, 1ull);
}

// classify()'s squared minimum-image gap between the boxes of tiles Iw and J — the same operations
// in the same order, so that k_tail_fix selects exactly the tile pairs the block kernel skipped
__device__ __forceinline__ double tile_gap2(const double* __restrict__ B, int T, int Iw, int J, double L, double invL) {
    double g2 = 0.;
#pragma unroll
    for (int c3 = 0; c3 < 3; ++c3) {
        double d = B[(size_t)c3 * T + Iw] - B[(size_t)c3 * T + J];
        d = fma(-__builtin_rint(d * invL), L, d);
        const double gap = fabs(d) - (B[(size_t)(3 + c3) * T + Iw] + B[(size_t)(3 + c3) * T + J]);
        g2 = gap > 0. ? fma(gap, gap, g2) : g2;
    }
    return g2;
}

// force_tail_mode 1, enforcement: for every listed tile I (its tail sum over eps) the exact sum of
// the pairs the skip radius dropped — every J tile whose box gap g satisfies r_t < g < L/2, all
// 64 x 64 pairs with the per-pair minimum image and the exact cutoff r < L/2 (SpeedUp:213-224) —
// is added to I's rows of `out` (F, or the rank's dense partial before the reduce-scatter).  Then
// each of I's ions has every pair inside L/2 (up to the far forms' own bounds).  One workgroup of
// 4 waves per listed tile (grid-stride over the list), wave q classifying the J tiles q*64 + l +
// 256 k lane-parallel and walking its ballot; the waves' sums combined in wave order: deterministic.
// Each ion belongs to one tile, so the read-modify-write of `out` has one writer.  With an empty
// list (the normal case) every workgroup reads st[3] and returns.
__global__ __launch_bounds__(256) void k_tail_fix(N3BArgs a, const unsigned long long* __restrict__ st,
                                                  const int* __restrict__ list, double* __restrict__ out) {
    __shared__ double part[4][3][64];
    const int n = (int)st[3];
    const int q = threadIdx.x >> 6, l = threadIdx.x & 63;
    const PairC c = {a.L, a.micT, a.micGuard, a.Rcut, a.lDeb, a.invlDeb, 1. / a.L, a.rc2, nullptr};
    const double rs2 = a.Rskip * a.Rskip, rcut2 = a.Rcut * a.Rcut;   // classify()'s rc2 and the tail test
    const int T = a.T, N = a.N, PS = a.Npad;
    for (int k = blockIdx.x; k < n; k += gridDim.x) {
        const int I = __builtin_amdgcn_readfirstlane(list[k]);
        const int i = I * 64 + l;
        const bool vi = i < N;
        const double xi = vi ? a.Rs[i] : 0., yi = vi ? a.Rs[PS + i] : 0., zi = vi ? a.Rs[2 * PS + i] : 0.;
        double fx = 0., fy = 0., fz = 0.;
        for (int j0 = q * 64; j0 < T; j0 += 256) {
            const int Jl = j0 + l;
            bool in = false;
            if (Jl < T) {
                const double g2 = tile_gap2(a.boxes, T, I, Jl, a.L, c.invL);
                in = g2 > rs2 && g2 < rcut2;
            }
            unsigned long long m = __ballot(in);
            while (m) {
                const int J = j0 + __builtin_ctzll(m);
                m &= m - 1;
                const int j = J * 64 + l;
                const int nj = min(64, N - J * 64);
                const double xl = j < N ? a.Rs[j] : 0., yl = j < N ? a.Rs[PS + j] : 0., zl = j < N ? a.Rs[2 * PS + j] : 0.;
                for (int t = 0; t < nj; ++t) {
                    auto lane_t = [t](double v) {
                        return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), t),
                                                __builtin_amdgcn_readlane(__double2loint(v), t));
                    };
                    double dx = xi - lane_t(xl), dy = yi - lane_t(yl), dz = zi - lane_t(zl);
                    mic_r(dx, dy, dz, c);
                    const double ft = pair_ft<1>(dx, dy, dz, c);   // 0 beyond L/2
                    fx = fma(dx, ft, fx); fy = fma(dy, ft, fy); fz = fma(dz, ft, fz);
                }
            }
        }
        part[q][0][l] = fx; part[q][1][l] = fy; part[q][2][l] = fz;
        __syncthreads();
        if (q == 0 && vi) {
            const int ion = a.perm[i];
            const int w = ion / a.S;
            double* o = out + (size_t)w * 3 * a.S + (ion - w * a.S);
#pragma unroll
            for (int c3 = 0; c3 < 3; ++c3) {
                const double v = ((part[0][c3][l] + part[1][c3][l]) + part[2][c3][l]) + part[3][c3][l];
                o[(size_t)c3 * a.S] += v;
            }
        }
        __syncthreads();
    }
}

// canonical per-ion sum of the slots this rank wrote: j-slots db = 0 .. nd-1, then i-slots.
// out: world 1 -> F [3][S]; sharded -> the rank's dense partial [world][3][S] (reduce-scattered)
__global__ __launch_bounds__(256) void k_n3b_reduce(N3BArgs a, double* __restrict__ out) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    const int k = blockIdx.y;
    if (g >= a.N) return;
    const int B = (g >> 6) / BW;
    const size_t plane = (size_t)3 * a.Npad;
    const double* p = a.slots + (size_t)k * a.Npad + g;
    double acc = 0.;
    for (int db = 0; db < a.nd; ++db) {
        const int P = (B - db + a.NB) % a.NB;
        const bool skip = !(a.NB & 1) && db == a.NB / 2 && P >= a.NB / 2;
        if (!skip && P >= a.Plo && P < a.Phi) acc = acc + p[(size_t)db * plane];
    }
    if (B >= a.Plo && B < a.Phi)
        for (int r = 0; r < a.R; ++r) acc = acc + p[(size_t)(a.nd + r) * plane];
    const int ion = a.use_sort ? a.perm[g] : g;     // spatial order: scatter back to the ion's place
    const int w = ion / a.S;
    out[(size_t)w * 3 * a.S + (size_t)k * a.S + (ion - w * a.S)] = acc;
}

// in-process rank group (tests): F of rank `rank` = sum over ranks r = 0.. of part[r]'s chunk
__global__ __launch_bounds__(256) void k_sum_rank_chunks(const double* const* parts, int world, int rank, int S,
                                                         double* __restrict__ F) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= 3 * S) return;
    double acc = 0.;
    for (int r = 0; r < world; ++r) acc = acc + parts[r][(size_t)rank * 3 * S + i];
    F[i] = acc;
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
static int seg_blocks(int nrows) { return (nrows + FT - 1) / FT; }

template <int MODE>
static hipError_t launch_rows(const ForceArgs& a, hipStream_t s) {
    if (a.nrows <= 0) return hipSuccess;
    dim3 grid(seg_blocks(a.nrows), a.nseg);
    if (a.variant == 1) {
        if (a.guard) hipLaunchKernelGGL((k_pairs<MODE, 1, true>), grid, dim3(FT), 0, s, a);
        else hipLaunchKernelGGL((k_pairs<MODE, 1, false>), grid, dim3(FT), 0, s, a);
    } else {
        if (a.guard) hipLaunchKernelGGL((k_pairs<MODE, 0, true>), grid, dim3(FT), 0, s, a);
        else hipLaunchKernelGGL((k_pairs<MODE, 0, false>), grid, dim3(FT), 0, s, a);
    }
    return hipGetLastError();
}

hipError_t launch_forces(const ForceArgs& a, hipStream_t s) { return launch_rows<0>(a, s); }
hipError_t launch_potential_rows(const ForceArgs& a, hipStream_t s) { return launch_rows<1>(a, s); }

hipError_t launch_reduce_segments(const double* Fpart, double* F, int nseg, int nrows, int S, int ncomp,
                                  hipStream_t s, size_t plane) {
    if (nrows <= 0) return hipSuccess;
    if (ncomp < 1 || ncomp > 3) return hipErrorInvalidValue;
    if (plane == 0) plane = (size_t)3 * S;
    if (plane < (size_t)ncomp * S) return hipErrorInvalidValue;
    dim3 grid((nrows + 255) / 256, ncomp);
    hipLaunchKernelGGL(k_reduce_segments, grid, dim3(256), 0, s, Fpart, F, nseg, nrows, S, ncomp, plane);
    return hipGetLastError();
}

hipError_t launch_forces_n3(const N3Args& a, int variant, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1) {
    if (a.npairs <= 0) return hipSuccess;
    dim3 grid(a.npairs);
#if defined(MDQT_EXPT_N3LDS)
    // diagnostic build only: extra dynamic LDS per workgroup (bytes) to cap workgroups per CU
    if (variant == 1 && !a.guard) {
        if (ev0) hipExtLaunchKernelGGL(k_pairs_n3<1, false>, grid, dim3(64 * N3W), MDQT_EXPT_N3LDS, s, ev0, ev1, 0, a);
        else hipLaunchKernelGGL((k_pairs_n3<1, false>), grid, dim3(64 * N3W), MDQT_EXPT_N3LDS, s, a);
        return hipGetLastError();
    }
#endif
    if (variant == 2) {
        if (a.guard) launch_timed(k_pairs_n3<2, true>, grid, dim3(64 * N3W), s, ev0, ev1, a);
        else launch_timed(k_pairs_n3<2, false>, grid, dim3(64 * N3W), s, ev0, ev1, a);
    } else if (variant == 1) {
        if (a.guard) launch_timed(k_pairs_n3<1, true>, grid, dim3(64 * N3W), s, ev0, ev1, a);
        else launch_timed(k_pairs_n3<1, false>, grid, dim3(64 * N3W), s, ev0, ev1, a);
    } else {
        if (a.guard) launch_timed(k_pairs_n3<0, true>, grid, dim3(64 * N3W), s, ev0, ev1, a);
        else launch_timed(k_pairs_n3<0, false>, grid, dim3(64 * N3W), s, ev0, ev1, a);
    }
    return hipGetLastError();
}

hipError_t launch_potential_n3(const N3Args& a, int variant, hipStream_t s) {
    if (a.npairs <= 0) return hipSuccess;
    if (variant < 0 || variant > 1) return hipErrorInvalidValue;
    const dim3 grid(a.npairs), blk(64 * N3W);
    if (variant == 1) {
        if (a.guard) hipLaunchKernelGGL((k_pairs_n3_pot<1, true>), grid, blk, 0, s, a);
        else hipLaunchKernelGGL((k_pairs_n3_pot<1, false>), grid, blk, 0, s, a);
    } else {
        if (a.guard) hipLaunchKernelGGL((k_pairs_n3_pot<0, true>), grid, blk, 0, s, a);
        else hipLaunchKernelGGL((k_pairs_n3_pot<0, false>), grid, blk, 0, s, a);
    }
    return hipGetLastError();
}

hipError_t launch_forces_n3b(const N3BArgs& a, int variant, double* out, hipStream_t s) {
    const int nblk = (a.Phi - a.Plo) * a.R;
    if (nblk > 0) {
        if (variant == 1) {
            if (a.guard) hipLaunchKernelGGL((k_pairs_n3b<1, true>), dim3(nblk), dim3(BW * 64), 0, s, a);
            else hipLaunchKernelGGL((k_pairs_n3b<1, false>), dim3(nblk), dim3(BW * 64), 0, s, a);
        } else {
            if (a.guard) hipLaunchKernelGGL((k_pairs_n3b<0, true>), dim3(nblk), dim3(BW * 64), 0, s, a);
            else hipLaunchKernelGGL((k_pairs_n3b<0, false>), dim3(nblk), dim3(BW * 64), 0, s, a);
        }
    }
    hipLaunchKernelGGL(k_n3b_reduce, dim3((a.N + 255) / 256, 3), dim3(256), 0, s, a, out);
    return hipGetLastError();
}

hipError_t launch_tail_max(const double* tailb, int T, double eps, int own_lo, int own_hi, unsigned long long* st,
                           int* list, hipStream_t s) {
    if (T <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_tail_max, dim3((T + 255) / 256 < 64 ? (T + 255) / 256 : 64), dim3(256), 0, s, tailb, T, eps,
                       own_lo, own_hi, st, list);
    return hipGetLastError();
}

hipError_t launch_tail_fix(const N3BArgs& a, const unsigned long long* st, const int* list, double* out,
                           hipStream_t s) {
    if (a.T <= 0 || !a.Rs || !a.perm || !a.boxes) return hipErrorInvalidValue;   // spatial order only
    hipLaunchKernelGGL(k_tail_fix, dim3(a.T < 512 ? a.T : 512), dim3(256), 0, s, a, st, list, out);
    return hipGetLastError();
}

hipError_t launch_potential_n3b(const N3BArgs& a, int variant, double* out, hipStream_t s) {
    if (variant < 0 || variant > 1) return hipErrorInvalidValue;
    const int nblk = (a.Phi - a.Plo) * a.R;
    if (nblk > 0) {
        if (variant == 1) {
            if (a.guard) hipLaunchKernelGGL((k_pairs_n3b<1, true, true>), dim3(nblk), dim3(BW * 64), 0, s, a);
            else hipLaunchKernelGGL((k_pairs_n3b<1, false, true>), dim3(nblk), dim3(BW * 64), 0, s, a);
        } else {
            if (a.guard) hipLaunchKernelGGL((k_pairs_n3b<0, true, true>), dim3(nblk), dim3(BW * 64), 0, s, a);
            else hipLaunchKernelGGL((k_pairs_n3b<0, false, true>), dim3(nblk), dim3(BW * 64), 0, s, a);
        }
    }
    hipLaunchKernelGGL(k_n3b_reduce, dim3((a.N + 255) / 256, 1), dim3(256), 0, s, a, out);   // component 0
    return hipGetLastError();
}

hipError_t launch_sum_rank_chunks(const double* const* parts, int world, int rank, int S, double* F, hipStream_t s) {
    hipLaunchKernelGGL(k_sum_rank_chunks, dim3((3 * S + 255) / 256), dim3(256), 0, s, parts, world, rank, S, F);
    return hipGetLastError();
}

}  // namespace mdqt
