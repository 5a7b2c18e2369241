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
#include <vector>
#include <cstdio>
#include "mdqt_internal.hpp"
#include "mdqt_pairs.hpp"

#include <math.h>
#include <type_traits>

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
// Newton-3 over BLOCK pairs (large N, one GPU or sharded): blocks of BW tiles (kN3BBlock: 8, 512
// ions; 16 until round 4); a workgroup of BW waves holds block P (wave q: tile I = BW P + q in registers) and walks the
// block distances db of its run, db in [0, NB/2] of the cyclic half shell (block Q = P + db mod
// NB; db = NB/2 only from P < NB/2 when NB is even; db = 0: tile pairs I <= J).  For every J
// tile of Q all 16 waves run their (I, J) rotation (64 steps; 32 on the diagonal tile) against
// the J tile in LDS with per-wave j accumulators, which are then combined in wave order and
// written to j-slot db (rows of J); each wave's i accumulator spans the whole run and goes to
// i-slot nd + run.  Slots: [nd + R][3][Npad], nd = NB/2 + 1 — O(N^2/1024) doubles, not O(N^2/64).
// The canonical per-ion sum (k_n3b_reduce) takes the j-slots in db order, then the i-slots in
// run order, skipping slots this rank does not write.
// ------------------------------------------------------------------------------------------
constexpr int BW = kN3BBlock;                       // tiles per block = waves per workgroup
#ifndef MDQT_N3B_AX1
#define MDQT_N3B_AX1 1                              // the one-axis per-pair image (n3b_pack_class); 0: all three axes
#endif
#ifndef MDQT_N3B_AX1_LEVELS
#define MDQT_N3B_AX1_LEVELS 0x1E                    // bit x: far level x takes it (1 mid, 2 far, 3 very far,
                                                    // 4 ultra far and its f32 level: the f64 ultra-far form, round 6)
#endif
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

// Sub-tile groups (round 4).  The J tile sits in LDS by 16-ion sub-tiles, each twice over: J ion
// 16 b + m at LDS index 32 b + m and 32 b + 16 + m (n3b_lds).  Lane l = 16 a + m (I sub-tile a) runs a
// tile pair as four groups of 16 steps: group d pairs I sub-tile a with J sub-tile (a + d) & 3 — a
// cyclic diagonal of the 4 x 4 sub-block matrix — and at step t lane l meets J ion
// 16 ((a + d) & 3) + ((m + t) & 15) at LDS index 32 ((a + d) & 3) + m + t (immediate offsets t).  A
// group covers its four sub-blocks once, and at every step the 64 lanes meet 64 distinct J ions (the
// j-side ds_add_f64 stays conflict-free).  Group d runs iff bit d of `groups` (wave-uniform): a group
// whose four sub-blocks all have sub-tile boxes farther apart than the skip radius is skipped — the
// pairs of a tile pair that straddles the cutoff sphere (or the tail radius) by less than a whole
// tile pair (tools/subtile_cull_model.py).  The diagonal tile (I = J): group 0 with
// t = 1..8 (t = 8 for m < 8 only: each pair inside a sub-tile once), group 1, and group 2 for a < 2
// (the sub-tile pairs (0, 2), (1, 3) once); group 3 would repeat group 1's pairs.
__device__ __forceinline__ int n3b_lds(int l) { return 32 * (l >> 4) + (l & 15); }   // J ion l's first copy

// The lane index recomputed where it is used (MDQT_N3B_REMAT): two VALU (v_mbcnt) in volatile asm, which
// the compiler neither hoists nor merges — so no VGPR holds the lane index, or a value derived from it,
// across the block kernel's J-step loop (at its 80-VGPR budget such values were spilled and reloaded
// with a vmcnt(0) wait at every pair-form dispatch)
#ifndef MDQT_N3B_REMAT
#define MDQT_N3B_REMAT 1
#endif
// One LDS-DMA load (global_load_lds_dwordx4: 16 bytes per lane from the lane's address g, into LDS at the
// wave-uniform byte offset lds + 16 x lane), in inline asm so that the compiler's wait-count pass does
// not see it: with the builtin it waited vmcnt(0) before every LDS atomic of the pair loops (a DMA
// writing LDS might alias them), retiring the DMA at once.  The caller counts and waits for it.
__device__ __forceinline__ void lds_dma16(const void* g, unsigned lds) {
    unsigned keep;
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}
template <typename T>
__device__ __forceinline__ unsigned lds_offset(T* p) {          // a __shared__ object's LDS byte offset
    return __builtin_amdgcn_readfirstlane((unsigned)(size_t)(__attribute__((address_space(3))) T*)p);
}
__device__ __forceinline__ int lane_opaque(int l) {
    if constexpr (!MDQT_N3B_REMAT) return l;
    int r;
    asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(r));
    return r;
}

// every 16 steps the LDS arrays are re-based at the lane's index (an opaque register), so the 16
// unrolled steps address them with immediate offsets t, 128 + t, 256 + t: without it the compiler's
// strength reduction moved the base past the arrays and spent a v_add_u32 per ds_add_f64 (3.5 VALU
// per pair, ~8 % of the block kernel's instructions)
#define N3B_REBASE(b0)                                                                     \
    int b_ = (b0);                                                                         \
    asm volatile("" : "+v"(b_));                                                           \
    const double (*pjb)[128] = (const double (*)[128])(&pj[0][0] + b_);                    \
    const double* mjb = mj + b_;                                                           \
    double *axb = ax + b_, *ayb = ay + b_, *azb = az + b_

// one sub-tile group: 16 rotation steps from LDS index b0 (the lane's first J ion) with weight w
template <int VARIANT, bool GUARD, bool RAGGED, bool SHIFT = false, bool CUT = VARIANT == 1 && MDQT_N3_CUT,
          bool POT = false, int FAR = 0, int NSTEP = 16, int MAX = -1>
__device__ __forceinline__ void n3b_group(int b0, double w, double xi, double yi, double zi, double mi,
                                          const double (*pj)[128], const double* mj, double* ax, double* ay,
                                          double* az, double& fx, double& fy, double& fz, const PairC& c,
                                          const double* nsh, double w_last = 1.) {
    N3B_REBASE(b0);
    if constexpr (MDQT_N3_DEFER_J) {
        // the j side one step late (n3_step_defer): each step's LDS reads queue behind the previous
        // step's atomics only one step later — the same adds in the same order, bit for bit
        double qx = 0., qy = 0., qz = 0.;
#pragma unroll
        for (int t = 0; t < NSTEP; ++t)
            n3_step_defer<VARIANT, GUARD, RAGGED, SHIFT, CUT, POT, FAR, MAX>(t, t == NSTEP - 1 ? w * w_last : w, xi, yi, zi,
                                                                             mi, pjb, mjb, axb, ayb, azb, fx, fy, fz, c,
                                                                             nsh, t - 1, qx, qy, qz);
        n3_j_add<POT>(NSTEP - 1, axb, ayb, azb, qx, qy, qz);
        return;
    }
    LdsPJ p = lds_pj(pjb, 0);
#pragma unroll
    for (int t = 0; t < NSTEP; ++t) {
        if constexpr (MDQT_LDS_SPLIT) {             // (the LDS bases opaque per step: ds_read_b64, no read2)
            lds_pj_opaque(p);
            n3_step<VARIANT, GUARD, RAGGED, SHIFT, CUT, POT, FAR, MAX, LdsPJ>(t, t == NSTEP - 1 ? w * w_last : w, xi, yi,
                                                                              zi, mi, p, mjb, axb, ayb, azb, fx, fy, fz,
                                                                              c, nsh);
        } else {
            n3_step<VARIANT, GUARD, RAGGED, SHIFT, CUT, POT, FAR, MAX>(t, t == NSTEP - 1 ? w * w_last : w, xi, yi, zi,
                                                                       mi, pjb, mjb, axb, ayb, azb, fx, fy, fz, c, nsh);
        }
    }
}

// a whole tile pair in one pair form: the groups of `groups` (off the diagonal) or the diagonal
// tile's three groups
template <int VARIANT, bool GUARD, bool RAGGED, bool SHIFT = false, bool CUT = VARIANT == 1 && MDQT_N3_CUT,
          bool POT = false, int FAR = 0, int MAX = -1>
__device__ __forceinline__ void n3b_pair(bool diag, unsigned groups, int l, double xi, double yi, double zi,
                                         double mi, const double (*pj)[128], const double* mj, double* ax,
                                         double* ay, double* az, double& fx, double& fy, double& fz,
                                         const PairC& c, const double* nsh = nullptr) {
    l = lane_opaque(l);
    const int a = l >> 4, m = l & 15;
    if (!diag) {
        for (int d = 0; d < 4; ++d) {
            if (!((groups >> d) & 1u)) continue;    // wave-uniform
            n3b_group<VARIANT, GUARD, RAGGED, SHIFT, CUT, POT, FAR, 16, MAX>(32 * ((a + d) & 3) + m, 1., xi, yi, zi, mi, pj,
                                                                             mj, ax, ay, az, fx, fy, fz, c, nsh);
        }
    } else if constexpr (MAX < 0) {                 // (a tile with itself has one image)
        // sub-tile distance 1..8 inside each sub-tile, the 8th once (m < 8)
        n3b_group<VARIANT, GUARD, RAGGED, SHIFT, CUT, POT, FAR, 8>(32 * a + m + 1, 1., xi, yi, zi, mi, pj, mj, ax, ay, az,
                                                                   fx, fy, fz, c, nsh, m >= 8 ? 0. : 1.);
        for (int d = 1; d < 3; ++d)
            n3b_group<VARIANT, GUARD, RAGGED, SHIFT, CUT, POT, FAR>(32 * ((a + d) & 3) + m, (d == 2 && a >= 2) ? 0. : 1.,
                                                                    xi, yi, zi, mi, pj, mj, ax, ay, az, fx, fy, fz, c, nsh);
    }
}

__device__ __forceinline__ float row_rol1f(float v) {   // lane 16 a + m <- lane 16 a + ((m + 1) & 15)
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x12F, 0xF, 0xF, false));   // row_ror:15
}

// An ultra-far tile pair (boxes >= r_ufar32 apart) with a uniform image, pair terms in f32
// (MDQT_UFAR32; error analysis and bound in mdqt_internal.hpp kUfar32A/B).  Round 5: the staging wave
// also holds the J tile in f32 relative to its first ion c_J (pj32 = fl32(xj - c_J)), the wave takes
// xi32 = fl32(xi - n L - c_J) once per tile pair and dx = fl32(xi32 - pj32) — no f64 subtraction and
// f32 conversion per pair — and (MDQT_UF32_PK) runs two rotation steps t, t + 1 through each packed
// instruction (v_pk_add_f32, v_pk_mul_f32, v_pk_fma_f32; v_rsq_f32, v_exp_f32 and the cutoff select
// per step): 16.75 VALU instructions per pair instead of 29.  The cutoff on the f32 r^2 (t = -inf).  The
// i side is summed in two f32 partials (even and odd steps), added, then added to the f64 partial; the j
// side is a running sum rotated one lane down inside the lane's row of 16 each step (row_ror:15 folded
// into the f32 add: lane m + 1's sum of the previous step is for lane m's current J ion; two steps at
// once: row_ror:14 of the sum plus row_ror:15 of step t's term plus step t + 1's) and ends in one
// ds_add_f64 per component at the group's last index.  Off the diagonal only (a tile's pair with
// itself is never ultra far).
static_assert(MDQT_SHIFT_I || !MDQT_UFAR32, "the f32 ultra-far form needs MDQT_SHIFT_I");
typedef float f32x2 __attribute__((ext_vector_type(2)));
__device__ __forceinline__ float row_rol2f(float v) {   // lane 16 a + m <- lane 16 a + ((m + 2) & 15)
    return __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), 0x12E, 0xF, 0xF, false));   // row_ror:14
}
// two rotation steps per v_pk_* instruction (MDQT_UF32_PK 1): gfx950 runs a packed f32 operation at half
// the rate of a scalar one (tools/ubench_f64: the same VALU cycles per pair) but issues half the
// instructions — A/B round 5 (profiles/r05h_uf32_force_ab.txt): C4 force call 244.8 ms packed, 248.3 scalar,
// 254.1 with the round-4 form (f64 separations); N = 1M 198.0 / 200.3 / 205.3.  0: one step at a time
#ifndef MDQT_UF32_PK
#define MDQT_UF32_PK 1
#endif

// POT (Epotential on the plan, round 6): u = 2^t ri in the same f32 operations, one component (i side in
// fx, j side in ax); its relative error is within the force form's (one factor ri instead of three)
template <bool POT = false>
__device__ __forceinline__ void n3b_group_uf32(int b0, float xi, float yi, float zi, const float (*pj32)[128],
                                               double* ax, double* ay, double* az, double& fx, double& fy, double& fz,
                                               float cf, float invlf, float rc2f) {
    // one opaque LDS address per component, so the 16 steps read them at immediate offsets (N3B_REBASE;
    // the array's own LDS offset and a shared base for the three components would not fit the
    // ds_read2_b32 offset field)
    typedef __attribute__((address_space(3))) const float* lds_f32p;
    lds_f32p px0 = (lds_f32p)&pj32[0][b0], py0 = (lds_f32p)&pj32[1][b0], pz0 = (lds_f32p)&pj32[2][b0];
    asm volatile("" : "+v"(px0), "+v"(py0), "+v"(pz0));
    if constexpr (POT) {
        f32x2 iu = {0.f, 0.f};
        float ju = 0.f;
#pragma unroll
        for (int t = 0; t < 16; t += 2) {
            const f32x2 dx = f32x2{xi, xi} - f32x2{px0[t], px0[t + 1]};
            const f32x2 dy = f32x2{yi, yi} - f32x2{py0[t], py0[t + 1]};
            const f32x2 dz = f32x2{zi, zi} - f32x2{pz0[t], pz0[t + 1]};
            const f32x2 r2 = __builtin_elementwise_fma(dx, dx, __builtin_elementwise_fma(dy, dy, dz * dz));
            const f32x2 ri = {__builtin_amdgcn_rsqf(r2.x), __builtin_amdgcn_rsqf(r2.y)};
            const f32x2 tt = (r2 * ri) * cf;
            const f32x2 e = {__builtin_amdgcn_exp2f(r2.x < rc2f ? tt.x : -INFINITY),
                             __builtin_amdgcn_exp2f(r2.y < rc2f ? tt.y : -INFINITY)};
            const f32x2 u = e * ri;
            const float uu = row_rol1f(u.x) + u.y;   // (the j side's rotation, as the forces')
            if (t == 0) { iu = u; ju = uu; }
            else { iu += u; ju = row_rol2f(ju) + uu; }
            asm volatile("" : "+v"(iu));
        }
        __hip_atomic_fetch_add(ax + b0 + 15, (double)ju, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        fx += (double)(iu.x + iu.y);
        (void)ay; (void)az; (void)fy; (void)fz; (void)invlf;
    } else if constexpr (MDQT_UF32_PK) {
        f32x2 ix = {0.f, 0.f}, iy = {0.f, 0.f}, iz = {0.f, 0.f};
        float jx = 0.f, jy = 0.f, jz = 0.f;
#pragma unroll
        for (int t = 0; t < 16; t += 2) {
            const f32x2 dx = f32x2{xi, xi} - f32x2{px0[t], px0[t + 1]};
            const f32x2 dy = f32x2{yi, yi} - f32x2{py0[t], py0[t + 1]};
            const f32x2 dz = f32x2{zi, zi} - f32x2{pz0[t], pz0[t + 1]};
            const f32x2 r2 = __builtin_elementwise_fma(dx, dx, __builtin_elementwise_fma(dy, dy, dz * dz));
            const f32x2 ri = {__builtin_amdgcn_rsqf(r2.x), __builtin_amdgcn_rsqf(r2.y)};
            const f32x2 tt = (r2 * ri) * cf;
            const f32x2 e = {__builtin_amdgcn_exp2f(r2.x < rc2f ? tt.x : -INFINITY),
                             __builtin_amdgcn_exp2f(r2.y < rc2f ? tt.y : -INFINITY)};
            const f32x2 ft = ((ri + invlf) * e) * (ri * ri);
            const f32x2 px = dx * ft, py = dy * ft, pz = dz * ft;
            // j side: S_t(m) = S_(t-1)(m + 1) + p_t(m); two steps: S_(t+1) = rol2(S_(t-1)) + (rol1(p_t) + p_(t+1))
            const float ux = row_rol1f(px.x) + px.y, uy = row_rol1f(py.x) + py.y, uz = row_rol1f(pz.x) + pz.y;
            if (t == 0) {
                ix = px; iy = py; iz = pz;
                jx = ux; jy = uy; jz = uz;
            } else {
                ix += px; iy += py; iz += pz;
                jx = row_rol2f(jx) + ux; jy = row_rol2f(jy) + uy; jz = row_rol2f(jz) + uz;
            }
            // each step pair's sums formed in their step pair (without it: 79 VGPRs spilled instead of 50)
            asm volatile("" : "+v"(ix), "+v"(iy), "+v"(iz));
        }
        const int b_ = b0;
        __hip_atomic_fetch_add(ax + b_ + 15, (double)jx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __hip_atomic_fetch_add(ay + b_ + 15, (double)jy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __hip_atomic_fetch_add(az + b_ + 15, (double)jz, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        fx += (double)(ix.x + ix.y); fy += (double)(iy.x + iy.y); fz += (double)(iz.x + iz.y);
    } else {
        float ix = 0.f, iy = 0.f, iz = 0.f, jx = 0.f, jy = 0.f, jz = 0.f;
#pragma unroll
        for (int t = 0; t < 16; ++t) {
            const float dx = xi - px0[t], dy = yi - py0[t], dz = zi - pz0[t];
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
                jx = row_rol1f(jx) + px; jy = row_rol1f(jy) + py; jz = row_rol1f(jz) + pz;
            }
            // each step's i and j sums formed in their step: without it the compiler sank the DPP adds
            // and the i-side adds after the last step and spilled the pending terms (80-VGPR budget)
            asm volatile("" : "+v"(ix), "+v"(iy), "+v"(iz));
        }
        const int b_ = b0;
        __hip_atomic_fetch_add(ax + b_ + 15, (double)jx, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __hip_atomic_fetch_add(ay + b_ + 15, (double)jy, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        __hip_atomic_fetch_add(az + b_ + 15, (double)jz, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_WAVEFRONT);
        fx += (double)ix; fy += (double)iy; fz += (double)iz;
    }
}

// the f32 ultra-far form over the groups of `groups` (off the diagonal); xi, yi, zi: the lane's ion
// relative to the J tile's raw box centre, in f32
template <bool POT = false>
__device__ __forceinline__ void n3b_pair_uf32(unsigned groups, int l, float xi, float yi, float zi,
                                              const float (*pj32)[128], double* ax, double* ay, double* az,
                                              double& fx, double& fy, double& fz, float cf, float invlf, float rc2f) {
    l = lane_opaque(l);
    const int a = l >> 4, m = l & 15;
    for (int d = 0; d < 4; ++d) {
        if (!((groups >> d) & 1u)) continue;        // wave-uniform
        n3b_group_uf32<POT>(32 * ((a + d) & 3) + m, xi, yi, zi, pj32, ax, ay, az, fx, fy, fz, cf, invlf, rc2f);
    }
}

// The class of tile pair (Iw, J) in spatial order (SpeedUp:222 keeps a pair only below r = L/2):
// returns the minimum-image multiples n_x, n_y, n_z of a uniform image and the class — skip when the
// boxes are farther apart than sqrt(r.rc2) (use_sort 1): -1 beyond L/2 (no pair inside the cutoff),
// -2 inside L/2 (the error-bounded tail: its pairs count in the tail sums) — else bit 0 = uniform
// image (FAST: the fast variant) + 2 x the far level (1 far, 2 very far, 3 ultra far, 4 ultra far in
// f32); g2 = the squared box gap.  Shared by k_pairs_n3b (the staging wave's lanes) and k_n3b_census.
struct N3BRadii { double rc2, rf2, rv2, ru2, ru32, rm2; };
// the squared radii of the classes: skip below the cutoff only for the forces (error-bounded tail,
// mdqt_engine.cpp tail_radius); the far forms are the fast force variant's
template <int VARIANT, bool POT>
__device__ __forceinline__ N3BRadii n3b_radii(const N3BArgs& a) {
    N3BRadii r;
    r.rc2 = POT ? a.Rcut * a.Rcut : a.Rskip * a.Rskip;
    r.rm2 = (POT || VARIANT != 1 || !MDQT_EXP_TAB || !(a.Rmid < a.Rcut)) ? INFINITY : a.Rmid * a.Rmid;
    r.rf2 = (POT || VARIANT != 1 || !(a.Rfar < a.Rcut)) ? INFINITY : a.Rfar * a.Rfar;
    r.rv2 = (POT || VARIANT != 1 || !(a.Rvfar < a.Rcut)) ? INFINITY : a.Rvfar * a.Rvfar;
    r.ru2 = (POT || VARIANT != 1 || !(a.Rufar < a.Rcut)) ? INFINITY : a.Rufar * a.Rufar;
    r.ru32 = (POT || VARIANT != 1 || !MDQT_UFAR32 || !(a.Rufar32 < a.Rcut)) ? INFINITY : a.Rufar32 * a.Rufar32;
    return r;
}
// the far level of a squared gap: 0 exact, 1 mid, 2 far, 3 very far, 4 ultra far, 5 ultra far in f32
__device__ __forceinline__ int n3b_level(double g2, const N3BRadii& r) {
    return g2 > r.ru32 ? 5 : g2 > r.ru2 ? 4 : g2 > r.rv2 ? 3 : g2 > r.rf2 ? 2 : g2 > r.rm2 ? 1 : 0;
}
// strad (when asked): bit c = axis c's minimum-image multiple varies over the tile pair's pairs
// (the core on two box columns: Bi = box column of Iw, Bj = of J, row stride ld — global [12][T], or the
// plan's LDS copy of its workgroup's tiles; the same operations in the same order either way)
template <bool FAST>
__device__ __forceinline__ double4 n3b_classify_p(const double* Bi, const double* Bj, int ld, double L, double invL,
                                                  double Rcut, int use_sort, const N3BRadii& r, double& g2,
                                                  int* strad = nullptr) {
    g2 = 0.;
    bool uni = true;
    int sm = 0;
    double n[3];
#pragma unroll
    for (int c3 = 0; c3 < 3; ++c3) {
        double d = Bi[c3 * ld] - Bj[c3 * ld];
        d = fma(-__builtin_rint(d * invL), L, d);
        const double gap = fabs(d) - (Bi[(3 + c3) * ld] + Bj[(3 + c3) * ld]);
        g2 = gap > 0. ? fma(gap, gap, g2) : g2;
        const double lo = Bi[(6 + c3) * ld] - Bj[(9 + c3) * ld];
        const double hi = Bi[(9 + c3) * ld] - Bj[(6 + c3) * ld];
        const double nlo = __builtin_rint(lo * invL), nhi = __builtin_rint(hi * invL);
        uni = uni && (nlo == nhi);
        sm |= (nlo == nhi ? 0 : 1) << c3;
        n[c3] = nlo;
    }
    if (strad) *strad = sm;
    const double cls = (use_sort == 1 && g2 > r.rc2) ? (g2 < Rcut * Rcut ? -2. : -1.)
                                                      : ((FAST && uni) ? 1. : 0.) + 2. * n3b_level(g2, r);
    return make_double4(n[0], n[1], n[2], cls);
}
template <bool FAST>
__device__ __forceinline__ double4 n3b_classify(const N3BArgs& a, double invL, const N3BRadii& r, int Iw, int J,
                                                double& g2, int* strad = nullptr) {
    return n3b_classify_p<FAST>(a.boxes + Iw, a.boxes + J, a.T, a.L, invL, a.Rcut, a.use_sort, r, g2, strad);
}

// the squared minimum-image gap between the boxes of 16-ion sub-tiles s and u ([6][T4] layout)
// (the core on two box columns Bs, Bu of row stride ld, as n3b_classify_p)
__device__ __forceinline__ double sub_gap2_p(const double* Bs, const double* Bu, int ld, double L, double invL) {
    double g2 = 0.;
#pragma unroll
    for (int c3 = 0; c3 < 3; ++c3) {
        double d = Bs[c3 * ld] - Bu[c3 * ld];
        d = fma(-__builtin_rint(d * invL), L, d);
        const double gap = fabs(d) - (Bs[(3 + c3) * ld] + Bu[(3 + c3) * ld]);
        g2 = gap > 0. ? fma(gap, gap, g2) : g2;
    }
    return g2;
}
__device__ __forceinline__ double sub_gap2(const double* __restrict__ SB, int T4, int s, int u, double L,
                                           double invL) {
    return sub_gap2_p(SB + s, SB + u, T4, L, invL);
}
// the sub-blocks (a, (a + d) & 3) of sub-tile group d as bits 4 a + b
constexpr unsigned kGroupBits[4] = {0x8421u, 0x1842u, 0x2184u, 0x4218u};
// each group's far level from the sub-blocks beyond r_mid / r_far / r_vfar / r_ufar / r_ufar32 (bit
// 4 a + b): the highest level all four of its sub-blocks reach, 4 bits per group (k_n3b_census: the
// same levels as k_n3b_plan's least group gap, counted another way)
__host__ __device__ __forceinline__ unsigned sub_group_levels(unsigned mm, unsigned mf, unsigned mv, unsigned mu,
                                                              unsigned m32) {
    unsigned lv = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d) {
        const unsigned g = kGroupBits[d];
        const unsigned x = (m32 & g) == g ? 5u : (mu & g) == g ? 4u : (mv & g) == g ? 3u : (mf & g) == g ? 2u
                         : (mm & g) == g ? 1u : 0u;
        lv |= x << (4 * d);
    }
    return lv;
}
// the groups of a staging word (n3b_stage_groups) that run in the pair form of far level x
__device__ __forceinline__ unsigned level_groups(unsigned word, int x) { return (word >> (4 + 4 * x)) & 15u; }
// the group mask of an off-diagonal tile pair from its 16 sub-block activities (bit 4 a + b: sub-tiles
// (a, b) closer than the skip radius): bit d = any sub-block (a, (a + d) & 3) active
__host__ __device__ __forceinline__ unsigned sub_groups_of(unsigned act16) {
    unsigned g = 0;
#pragma unroll
    for (int d = 0; d < 4; ++d)
#pragma unroll
        for (int a = 0; a < 4; ++a) g |= ((act16 >> (4 * a + ((a + d) & 3))) & 1u) << d;
    return g;
}
// one pair's |F| bound at distance >= the gap d (g2 = d^2 > 0): g(d) = (1/d + 1/lDeb) e^(-d/lDeb) / d
// (SpeedUp:224 times r), the tail sums' term, as an upper bound in a few f32 operations: v_rsq_f32
// and v_exp_f32 (each within 2^-22 relative, tests/test_gpu_large.py), d^2 and the exponent's
// constant rounded to f32 (e^(-d/lDeb) within (d/lDeb) 2^-23 relative), the result x (1 + 2^-12):
// an upper bound while d/lDeb < 1000; beyond f32's range e^(-d/lDeb) flushes to 0 (< 1e-44)
__device__ __forceinline__ double tail_g(double g2, float invl, float cf) {
    const float s = (float)g2;
    const float ri = __builtin_amdgcn_rsqf(s);
    const float e = __builtin_amdgcn_exp2f((s * ri) * cf);
    return (double)(((ri + invl) * e) * ri) * (1. + 0x1p-12);
}
// force_form_mode 1: the bound on the error of one pair term at distance >= the gap d (g2 = d^2) in the
// pair form of level e >= 1: g(d) err_e(d) = g(d) (kFormErrA[e] d/lDeb + kFormErrB[e]) — both factors as
// upper bounds in f32 (tail_g's; d/lDeb within 3 2^-23), the product x (1 + 2^-10).  g err_e decreases
// in d for every form (its log-derivative is below 1/(1 + x) - 1/x - 1 < 0, x = d/lDeb), so each of the
// sub-block's pairs (distance >= its gap) is bounded by it.
// (the constants rounded up to f32; the whole term in f32 — f32 VALU issues at twice the f64 rate — and
// x (1 + 2^-10) covers every rounding: tail_g's 2^-12 bound, d/lDeb's 3 2^-23, the err factor's and the
// product's 2^-23 each)
__constant__ const float kFormA[6] = {(float)kFormErrA[0], (float)(kFormErrA[1] * (1. + 0x1p-20)),
                                      (float)kFormErrA[2], (float)(kFormErrA[3] * (1. + 0x1p-20)),
                                      (float)(kFormErrA[4] * (1. + 0x1p-20)), (float)(kFormErrA[5] * (1. + 0x1p-20))};
__constant__ const float kFormB[6] = {(float)kFormErrB[0], (float)(kFormErrB[1] * (1. + 0x1p-20)),
                                      (float)(kFormErrB[2] * (1. + 0x1p-20)), (float)(kFormErrB[3] * (1. + 0x1p-20)),
                                      (float)(kFormErrB[4] * (1. + 0x1p-20)), (float)(kFormErrB[5] * (1. + 0x1p-20))};
__device__ __forceinline__ double form_term(double g2, float invl, float cf, int e) {
    const float s = (float)g2;
    const float ri = __builtin_amdgcn_rsqf(s);
    const float r = s * ri;
    const float ex = __builtin_amdgcn_exp2f(r * cf);
    const float g = ((ri + invl) * ex) * ri;
    return (double)(g * fmaf(r * invl, kFormA[e], kFormB[e])) * (1. + 0x1p-10);
}
// force_form_mode 1: an upper bound on the squared distance of any pair of boxes s and u in the minimum
// image — a uniform-image tile pair's pairs are each at their minimum image in the block kernel (its shift
// is every pair's rint(dx / L)), and per axis min_k |x_i - x_j - k L| <= |mi(c_s - c_u)| + h_s + h_u, whatever
// frame the boxes' centres were taken in (a box is the min / max about its first ion, k_tile_boxes)
__device__ __forceinline__ double sub_far2_p(const double* Bs, const double* Bu, int ld, double L, double invL) {
    double f2 = 0.;
#pragma unroll
    for (int c3 = 0; c3 < 3; ++c3) {
        double d = Bs[c3 * ld] - Bu[c3 * ld];
        d = fma(-__builtin_rint(d * invL), L, d);
        const double f = fabs(d) + (Bs[(3 + c3) * ld] + Bu[(3 + c3) * ld]);
        f2 = fma(f, f, f2);
    }
    return f2;
}
__device__ __forceinline__ double sub_far2(const double* __restrict__ SB, int T4, int s, int u, double L, double invL) {
    return sub_far2_p(SB + s, SB + u, T4, L, invL);
}
// a tile pair's class and uniform-image multiples in one LDS word: bits 0-3 class + 2, 4-11 / 12-19 /
// 20-27 n_x, n_y, n_z (signed); a uniform image with a multiple beyond +-127 (positions that far
// outside the box) is taken per pair instead.  A per-pair image that varies on ONE axis only (strad:
// n3b_classify's mask; FAST) carries that axis + 1 in bits 28-29 and the other two axes' multiples
// (the varying axis's field 0): the block kernel then takes the minimum image per pair on that axis
// alone (the tile pairs that straddle the image boundary, ~97 % of the per-pair-image ones, C3/C5)
__device__ __forceinline__ int n3b_pack_class(double4 t4, int strad = 0) {
    int cls = (int)t4.w;
    const bool uni = cls >= 0 && (cls & 1);
    if (uni && !(fabs(t4.x) <= 127. && fabs(t4.y) <= 127. && fabs(t4.z) <= 127.)) cls -= 1;
    const bool u2 = cls >= 0 && (cls & 1);
    const int ax1 = strad == 1 ? 1 : strad == 2 ? 2 : strad == 4 ? 3 : 0;
    const bool one = MDQT_N3B_AX1 && cls >= 0 && !(cls & 1) && ax1 &&
                     fabs(t4.x) <= 127. && fabs(t4.y) <= 127. && fabs(t4.z) <= 127.;
    const int nx = (u2 || (one && ax1 != 1)) ? (int)t4.x : 0, ny = (u2 || (one && ax1 != 2)) ? (int)t4.y : 0,
              nz = (u2 || (one && ax1 != 3)) ? (int)t4.z : 0;
    return (cls + 2) | ((nx & 255) << 4) | ((ny & 255) << 12) | ((nz & 255) << 20) | ((one ? ax1 : 0) << 28);
}
// real ions of 16-ion sub-tile s (0 for the padding of the ragged last tile)
__device__ __forceinline__ double sub_count(int N, int s) { return (double)max(0, min(16, N - 16 * s)); }
// tile J's raw box (the exact min / max of its coordinates, boxes [6, 12)): its squared half-diagonal —
// the f32 ultra-far form (n3b_group_uf32) stages J relative to J's first ion and takes a sub-tile group
// only where the box diagonal (twice this) is within the group's gap (kUfar32A/B's premise)
__device__ __forceinline__ double raw_half2_p(const double* Bj, int ld) {
    double h2 = 0.;
#pragma unroll
    for (int c3 = 0; c3 < 3; ++c3) {
        const double h = 0.5 * (Bj[(9 + c3) * ld] - Bj[(6 + c3) * ld]);
        h2 = fma(h, h, h2);
    }
    return h2;
}
__device__ __forceinline__ double raw_half2(const double* B, int T, int J) { return raw_half2_p(B + J, T); }


// One tile pair (I, J) of the block kernels (k_pairs_n3b, k_pairs_n3b_pw): its sub-tile groups of `word`
// (k_n3b_plan) in the pair forms of their levels, the image of the class word `tw` (n3b_pack_class); the i
// side into tx, ty, tz (a fresh sum per tile pair), the j side into the wave's accumulators ax, ay, az.
// rag: the ragged last tile is one of the two (exact form, validity weights)
template <int VARIANT, bool GUARD, bool POT, bool AXP>
__device__ __forceinline__ void n3b_tile_pair(const N3BArgs& a, const PairC& c, int l, bool diag, bool rag, int tw,
                                              unsigned word, double xi, double yi, double zi, double mi,
                                              const double (*pj)[128], const double* mj, const float (*pj32)[128],
                                              double* ax, double* ay, double* az, double& tx, double& ty, double& tz,
                                              float cf32, float invl32, float rc2f) {
    constexpr bool CUT = VARIANT == 1 && MDQT_N3_CUT;
    constexpr bool FARF = VARIANT == 1 && !GUARD && CUT;   // the error-bounded pair forms
    const unsigned groups = word & 15u;
    const int ci = (tw & 15) - 2;       // bit 0 uniform image (the tile pair's)
    if (rag)
        n3b_pair<VARIANT, GUARD, true, false, CUT, POT>(diag, groups, l, xi, yi, zi, mi, pj, mj, ax, ay,
                                                        az, tx, ty, tz, c);
    else if (VARIANT == 1 && (ci & 1)) {       // uniform image
        const double nsh[3] = {(double)((tw << 20) >> 24), (double)((tw << 12) >> 24), (double)((tw << 4) >> 24)};
        // xi - n L once per tile pair (n3_step SHIFT; MDQT_SHIFT_I)
        const double sx = MDQT_SHIFT_I ? fma(-nsh[0], a.L, xi) : xi;
        const double sy = MDQT_SHIFT_I ? fma(-nsh[1], a.L, yi) : yi;
        const double sz = MDQT_SHIFT_I ? fma(-nsh[2], a.L, zi) : zi;
        if constexpr (FARF) {
            if (diag) {                 // (a tile with itself: the exact form)
                n3b_pair<VARIANT, GUARD, false, true, CUT, POT>(true, groups, l, sx, sy, sz, mi, pj, mj, ax, ay,
                                                                az, tx, ty, tz, c, nsh);
            } else {                    // each form over the groups at its level
                const unsigned g5 = level_groups(word, 5), g4 = level_groups(word, 4),
                               g3 = level_groups(word, 3), g2 = level_groups(word, 2),
                               g1 = level_groups(word, 1), g0 = level_groups(word, 0);
                if (g4) n3b_pair<VARIANT, GUARD, false, true, CUT, POT, 4>(false, g4, l, sx, sy, sz, mi, pj, mj,
                                                                           ax, ay, az, tx, ty, tz, c, nsh);
                if (g3) n3b_pair<VARIANT, GUARD, false, true, CUT, POT, 3>(false, g3, l, sx, sy, sz, mi, pj, mj,
                                                                           ax, ay, az, tx, ty, tz, c, nsh);
                if (g2) n3b_pair<VARIANT, GUARD, false, true, CUT, POT, 2>(false, g2, l, sx, sy, sz, mi, pj, mj,
                                                                           ax, ay, az, tx, ty, tz, c, nsh);
                if (MDQT_EXP_TAB && g1)
                    n3b_pair<VARIANT, GUARD, false, true, CUT, POT, MDQT_EXP_TAB ? 1 : 0>(
                        false, g1, l, sx, sy, sz, mi, pj, mj, ax, ay, az, tx, ty, tz, c, nsh);
                if (g0) n3b_pair<VARIANT, GUARD, false, true, CUT, POT>(false, g0, l, sx, sy, sz, mi, pj, mj, ax,
                                                                        ay, az, tx, ty, tz, c, nsh);
#if !defined(MDQT_EXPT_UFAR_SKIP)                   // last: nothing after it keeps sx, nsh live (diagnostic build: skip it, wrong results)
                if (g5) n3b_pair_uf32<POT>(g5, l, (float)(sx - pj[0][0]), (float)(sy - pj[1][0]),
                                           (float)(sz - pj[2][0]), pj32, ax, ay, az, tx, ty, tz, cf32,
                                           invl32, rc2f);
#endif
            }
        } else {
            n3b_pair<VARIANT, GUARD, false, VARIANT == 1, CUT, POT>(diag, groups, l, sx, sy, sz, mi, pj, mj,
                                                                    ax, ay, az, tx, ty, tz, c, nsh);
        }
    } else if constexpr (FARF) {       // per-pair image
        const int ax1 = (tw >> 28) & 3;  // 1 + the one axis whose image varies (n3b_pack_class)
        if (diag) {
            n3b_pair<VARIANT, GUARD, false, false, CUT, POT>(true, groups, l, xi, yi, zi, mi, pj, mj, ax, ay,
                                                             az, tx, ty, tz, c);
        } else if (AXP && ax1) {        // one axis: the other two shifted once (xi - n L)
          if constexpr (AXP) {
            const double sx = fma(-(double)((tw << 20) >> 24), a.L, xi);   // (0 on the varying axis:
            const double sy = fma(-(double)((tw << 12) >> 24), a.L, yi);   //  fma(-0, L, x) = x)
            const double sz = fma(-(double)((tw << 4) >> 24), a.L, zi);
            constexpr unsigned LV = MDQT_N3B_AX1_LEVELS;   // the levels that take it (bit x: level x)
            // (levels 4 and 5 in the f64 ultra-far form with the one-axis image — the f32 form needs a
            // uniform image; without LV bit 4 they ride in the very-far form)
            const unsigned g45 = level_groups(word, 4) | level_groups(word, 5);
            const unsigned g3 = level_groups(word, 3) | ((LV & 16u) ? 0u : g45), g4 = (LV & 16u) ? g45 : 0u,
                           g2 = level_groups(word, 2), g1 = level_groups(word, 1), g0 = level_groups(word, 0);
            auto one_axis = [&](auto axc) {
                constexpr int AX = decltype(axc)::value;
                if ((LV & 16u) && g4)
                    n3b_pair<VARIANT, GUARD, false, false, CUT, POT, 4, AX>(false, g4, l, sx, sy, sz, mi, pj, mj,
                                                                            ax, ay, az, tx, ty, tz, c);
                if ((LV & 8u) && g3)
                    n3b_pair<VARIANT, GUARD, false, false, CUT, POT, 3, AX>(false, g3, l, sx, sy, sz, mi, pj, mj,
                                                                            ax, ay, az, tx, ty, tz, c);
                if ((LV & 4u) && g2)
                    n3b_pair<VARIANT, GUARD, false, false, CUT, POT, 2, AX>(false, g2, l, sx, sy, sz, mi, pj, mj,
                                                                            ax, ay, az, tx, ty, tz, c);
                if ((LV & 2u) && MDQT_EXP_TAB && g1)
                    n3b_pair<VARIANT, GUARD, false, false, CUT, POT, MDQT_EXP_TAB ? 1 : 0, AX>(
                        false, g1, l, sx, sy, sz, mi, pj, mj, ax, ay, az, tx, ty, tz, c);
            };
            if (ax1 == 1) one_axis(std::integral_constant<int, 0>{});
            else if (ax1 == 2) one_axis(std::integral_constant<int, 1>{});
            else one_axis(std::integral_constant<int, 2>{});
            // the other levels per pair (the exact level with a varying image: ~never, C3 1.6e-5
            // of the pairs)
            if (!(LV & 8u) && g3)
                n3b_pair<VARIANT, GUARD, false, false, CUT, POT, 3>(false, g3, l, xi, yi, zi, mi, pj, mj, ax, ay,
                                                                    az, tx, ty, tz, c);
            if (!(LV & 4u) && g2)
                n3b_pair<VARIANT, GUARD, false, false, CUT, POT, 2>(false, g2, l, xi, yi, zi, mi, pj, mj, ax, ay,
                                                                    az, tx, ty, tz, c);
            if (!(LV & 2u) && MDQT_EXP_TAB && g1)
                n3b_pair<VARIANT, GUARD, false, false, CUT, POT, MDQT_EXP_TAB ? 1 : 0>(
                    false, g1, l, xi, yi, zi, mi, pj, mj, ax, ay, az, tx, ty, tz, c);
            if (g0) n3b_pair<VARIANT, GUARD, false, false, CUT, POT>(false, g0, l, xi, yi, zi, mi, pj, mj, ax,
                                                                     ay, az, tx, ty, tz, c);
          }
        } else {                        // (ultra far with a per-pair image: rare, very-far form)
            const unsigned g3 = level_groups(word, 3) | level_groups(word, 4) | level_groups(word, 5),
                           g2 = level_groups(word, 2), g1 = level_groups(word, 1), g0 = level_groups(word, 0);
            if (g3) n3b_pair<VARIANT, GUARD, false, false, CUT, POT, 3>(false, g3, l, xi, yi, zi, mi, pj, mj, ax,
                                                                        ay, az, tx, ty, tz, c);
            if (g2) n3b_pair<VARIANT, GUARD, false, false, CUT, POT, 2>(false, g2, l, xi, yi, zi, mi, pj, mj, ax,
                                                                        ay, az, tx, ty, tz, c);
            if (MDQT_EXP_TAB && g1)
                n3b_pair<VARIANT, GUARD, false, false, CUT, POT, MDQT_EXP_TAB ? 1 : 0>(false, g1, l, xi, yi, zi, mi,
                                                                                   pj, mj, ax, ay, az, tx, ty, tz, c);
            if (g0) n3b_pair<VARIANT, GUARD, false, false, CUT, POT>(false, g0, l, xi, yi, zi, mi, pj, mj, ax, ay,
                                                                     az, tx, ty, tz, c);
        }
    } else
        n3b_pair<VARIANT, GUARD, false, false, CUT, POT>(diag, groups, l, xi, yi, zi, mi, pj, mj, ax, ay, az,
                                                         tx, ty, tz, c);
}

// POT: Epotential's pair potential (component 0 of the slots, both rows +u) instead of the force
// the fast variant fits 80 VGPRs (6 waves per SIMD: three 8-wave workgroups per CU); the exact one (libm exp, divisions) gets 128
#ifndef MDQT_N3B_IRUN_LDS
#define MDQT_N3B_IRUN_LDS 1                         // the run's i accumulator in LDS (0: in the i-slot itself)
#endif
#ifndef MDQT_N3B_WPE                                // waves per SIMD of the fast variant (VGPR budget 512/WPE):
#define MDQT_N3B_WPE (BW == 8 ? 6 : 8)              // 6 = three 8-wave workgroups per CU (41.5 KB LDS each)
#endif
// double-buffered J staging by LDS-DMA (plan path), one step ahead.  Measured (round 5, force-call A/B,
// 2 alternations, tools/gpu/r05_ab.sh): slower than the synchronous staging — C3 6.585 vs 6.54 ms, C5
// 31.93 vs 31.73, N = 1M 205.1 vs 203.0: the J-step barrier wait is the waves' unequal pair work, not
// the staging load.  Off by default, kept as an option
#ifndef MDQT_N3B_DBUF
#define MDQT_N3B_DBUF 0
#endif
static_assert(!(MDQT_N3B_DBUF && MDQT_UFAR32), "the double-buffered staging has no f32 J copy: build it with MDQT_UFAR32 0");
// the block kernel's LDS, one object (k_pairs_n3b)
constexpr int kN3BStageBufs = MDQT_N3B_DBUF ? 2 : 1;
template <int W>
struct N3BShared {
    double pj[kN3BStageBufs][3][128];               // J positions by sub-tiles twice over (n3b_lds), per buffer
    float pj32[3][128];                             // the same, fl32(xj - c_J), c_J = J's first ion (the f32 ultra-far form)
    double accj[W][3][128];                         // per-wave j accumulators
    double mjs[2][128];                             // J validity weights: all ones / the ragged last tile's
    double etab[64];                                // 2^(k/64) (MDQT_EXP_TAB)
#if MDQT_N3B_IRUN_LDS
    double irun[W][3][64];                          // the run's i accumulators
#endif
    uint2 pw[kN3BStageBufs][W];                     // plan words (class, sub-tile groups), per buffer
};
// AXP: the one-axis per-pair image (n3b_pack_class bits 28-29) in an instance of its own, launched
// only where such tile pairs can lie inside the skip radius (launch_forces_n3b): compiled into the
// one instance it cost the calls without any (N = 1M) 0.5 %.
template <int VARIANT, bool GUARD, bool POT = false, bool AXP = false>
__global__ __launch_bounds__(BW * 64) __attribute__((amdgpu_waves_per_eu(VARIANT == 1 ? MDQT_N3B_WPE : 4, VARIANT == 1 ? MDQT_N3B_WPE : 4)))
void k_pairs_n3b(N3BArgs a) {
    // all LDS in one object: beside an LDS-DMA (the plan path's J staging) a second __shared__ object
    // can make the compiler wait for the DMA before unrelated LDS reads (cdna_hip_programming.md §5)
    __shared__ N3BShared<BW> sh;
    double* const etab = sh.etab;
    stage_exp_tab(etab);
    const int q = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;   // q: wave-uniform
    const int l0 = l;                               // (lane_opaque's fallback)
#ifndef MDQT_N3B_ORDER
#define MDQT_N3B_ORDER 1
#endif
    // workgroup order: run-major (MDQT_N3B_ORDER 1) dispatches every block's first run — the near
    // block distances, the heaviest work — first and the far, mostly skipped runs last, so the
    // kernel's last round is short; 0: block-major (round 3)
    const int nP = a.Phi - a.Plo;
    const int P = a.Plo + (MDQT_N3B_ORDER ? (int)blockIdx.x % nP : (int)blockIdx.x / a.R);
    const int run = MDQT_N3B_ORDER ? (int)blockIdx.x / nP : (int)blockIdx.x % a.R;
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
    // waited for here, once: as load results the compiler waited vmcnt(0) for them at every pair-form
    // dispatch (it cannot count past the staging wave's LDS-DMA on the loop's back edge), which retired
    // the DMA just issued instead of letting it land during the pair work
    asm volatile("" : "+v"(xi), "+v"(yi), "+v"(zi));
    // Tile-pair classes in spatial order (SpeedUp:222 keeps a pair only below r = L/2), decided
    // for all BW waves' tile pairs (I, J) by the staging wave's lanes 0..BW-1:
    //  * skip (force_sort 1): boxes beyond the skip radius in the minimum image — at L/2 no pair
    //    inside the cutoff (exact zeros), inside L/2 the error-bounded tail (tail sums below);
    //  * uniform image: every pair's raw separation fl(xi - xj) lies in [fl(lo_I - hi_J),
    //    fl(hi_I - lo_J)] (rounding is monotone), and so does rint(fl(dx / L)) between the rints
    //    of the two ends; equal ends = one minimum-image multiple per axis for every pair, bit for
    //    bit what mic_r computes per pair (the fast variant then skips that rint per pair);
    //  * otherwise the per-pair minimum image.
    // class: -1 / -2 skip; otherwise bit 0 = uniform image, + 2 x the far level (n3b_level: 1 mid, 2
    // far, 3 very far, 4 ultra far, 5 ultra far in f32; forces only): 0 .. 11 (n3b_pack_class: tpw[q]).
    // The forces take them, with the sub-tile groups (tg[q]), from the call's plan (k_n3b_plan: one
    // 8-byte word per tile pair, loaded by lanes 0..15); without a plan (potentials, unsorted order)
    // the staging lanes classify the tile pairs themselves and every group runs in the exact form.
    constexpr bool CUT = VARIANT == 1 && MDQT_N3_CUT;
    constexpr bool FARF = VARIANT == 1 && !GUARD && CUT;   // the error-bounded pair forms (potentials: on a plan)
    const N3BRadii rad = n3b_radii<VARIANT, POT>(a);
    // the f32 form's constants as wave-uniform SGPR values (in VGPRs they were spilled and reloaded
    // inside the pair loop at the kernel's 64-VGPR budget)
    auto sgpr_f = [](float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); };
    const float cf32 = sgpr_f((float)(a.invlDeb * kNegLog2e)), invl32 = sgpr_f((float)a.invlDeb),
                rc2f = sgpr_f((float)a.rc2);
    // the run's i accumulator: in LDS (read and written once per block distance, so that the
    // three-level blocking fits the 64-VGPR budget), or (MDQT_N3B_IRUN_LDS 0) the i-slot itself —
    // each wave's own rows, read, added and written once per block distance, in order
#if MDQT_N3B_IRUN_LDS
    auto fiptr = [&]() { return sh.irun[q][0] + lane_opaque(l0); };
    constexpr size_t FS = 64;
#else
    auto fiptr = [&]() { return a.slots + (size_t)(a.nd + run) * ((size_t)3 * a.Npad) + I * 64 + lane_opaque(l0); };
    const size_t FS = a.Npad;
#endif
    bool fi_first = true;
    const uint2* plan = a.plan;                     // (potentials: the plan of launch_potential_n3b, or none)
    // every J step: the staging wave (the last; not one of the combining waves 0..2) loads J, one
    // barrier, the pair work, one barrier, then waves 0..2 combine the 16 j accumulators of one
    // component each into the j-slot and zero them for the next step — while the staging wave
    // already loads the next J (no third barrier: nothing reads pj or the plan words after the
    // second, and the accumulators are zero again before the combining waves reach the next one)
    constexpr int kStage = BW - 1;
#pragma unroll
    for (int k = 0; k < 3; ++k) { sh.accj[q][k][l] = 0.; sh.accj[q][k][l + 64] = 0.; }
    double* ax = sh.accj[q][0];
    double* ay = sh.accj[q][1];
    double* az = sh.accj[q][2];
    // the J tile's validity weights (RAGGED pair steps): all ones, or the ragged last tile's pattern —
    // constant over the launch, written once (a J tile takes mjs[J == T - 1])
    if (q == kStage) {
        const int li = n3b_lds(l);
        const double m1 = (T - 1) * 64 + l < N ? 1. : 0.;
        sh.mjs[0][li] = 1.; sh.mjs[0][li + 16] = 1.;
        sh.mjs[1][li] = m1; sh.mjs[1][li + 16] = m1;
    }
    const size_t plane = (size_t)3 * a.Npad;
    // the plan's J-step masks (after its tile-pair words): bit b = some tile pair of J step b has work
    const unsigned* jsteps = plan ? (const unsigned*)(plan + (size_t)(a.Phi - a.Plo) * a.nd * (BW * BW)) : nullptr;
    auto half_db = [&](int db) { return !(a.NB & 1) && db == a.NB / 2 && P >= a.NB / 2; };   // the other half covers it
    // Double-buffered J staging (MDQT_N3B_DBUF, the plan path): at the top of every J step with work the
    // staging wave issues the LDS-DMA loads (global_load_lds_dwordx4: J's positions by sub-tiles twice
    // over, and the step's 8 plan words) of the NEXT step with work into the other buffer, then all waves
    // compute on this one; the DMA lands during the pair work and is retired by the staging wave's wait
    // at the step's second barrier.  The first barrier is a raw s_barrier after lgkmcnt(0) (the
    // combine's zeroing), so the DMA in flight is not drained there.  Without a plan (potentials,
    // unsorted order) the staging wave loads and classifies J itself before the first barrier.
    // Rs holds the pad ions' values (k_gather_sorted), so the DMA copies what the register path computes.
    constexpr bool kDbuf = MDQT_N3B_DBUF != 0;
    int buf = 0;
    auto next_step = [&](int db, int b, int& odb, int& ob) {   // the first step with work at or after (db, b)
        for (; db < d1; ++db, b = 0) {
            if (half_db(db)) continue;
            const unsigned msk = jsteps[2 * ((size_t)(P - a.Plo) * a.nd + db)];
            const int Qn = (P + db) % a.NB;
            for (; b < BW && Qn * BW + b < T; ++b)
                if ((msk >> b) & 1u) { odb = db; ob = b; return; }
        }
        odb = d1; ob = 0;
    };
    auto dma_stage = [&](int bf, int db, int b) {   // (staging wave) J step (db, b) into buffer bf
        const int J = ((P + db) % a.NB) * BW + b;
        const int l = lane_opaque(l0);
        const double* src = a.Rs + (size_t)J * 64 + 16 * (l >> 4) + ((2 * l) & 15);
        // lanes 0 .. BW/2 - 1: the step's BW plan words, 16 bytes each (an LDS-DMA writes base + 16 x lane
        // for every active lane, so only those lanes issue it)
        const uint2* pws = plan + ((size_t)(P - a.Plo) * a.nd + db) * (BW * BW) + b * BW + 2 * (l & (BW / 2 - 1));
        // every address formed before the first DMA: a spill reload between them would be waited for
        // with vmcnt(0), retiring the DMA already issued
        asm volatile("" : "+v"(src), "+v"(pws));
        if (l < BW / 2) lds_dma16(pws, lds_offset(&sh.pw[bf][0]));
#pragma unroll
        for (int c3 = 0; c3 < 3; ++c3) lds_dma16(src + (size_t)c3 * a.Npad, lds_offset(&sh.pj[bf][c3][0]));
    };
    if (kDbuf && plan && q == kStage) {             // the launch's first step with work into buffer 0
        int fdb, fb;
        next_step(d0, 0, fdb, fb);
        if (fdb < d1) dma_stage(0, fdb, fb);
    }
    for (int db = d0; db < d1; ++db) {
        if (half_db(db)) continue;
        const int Q = (P + db) % a.NB;
        double bx = 0., by = 0., bz = 0.;          // this block distance's i partial (3-level blocking)
        // the block distance's J-step mask, read once and held in an SGPR (wave-uniform; read per J step
        // it was a vector load and a vmcnt(0) wait at the top of every step)
        const unsigned jmask = jsteps ? __builtin_amdgcn_readfirstlane(jsteps[2 * ((size_t)(P - a.Plo) * a.nd + db)]) : ~0u;
        for (int b = 0; b < BW; ++b) {
            const int J = Q * BW + b;
            if (J >= T) break;
            if (jsteps && !((jmask >> b) & 1u)) {   // every tile pair of this J step skipped (wave-uniform):
                if (q < (POT ? 1 : 3) && !a.tmask)  // J's rows get the combine's value, -0, and no barrier (with
                    a.slots[(size_t)db * plane + (size_t)q * a.Npad + J * 64 + lane_opaque(l0)] = POT ? 0. : -0.;
                continue;                           // the reduction's masks: nothing, the slot is not read)
            }
            if (kDbuf && plan) {
                if (q == kStage) {                  // the next step with work into the other buffer
                    int ndb, nb;
                    next_step(db, b + 1, ndb, nb);
                    // this buffer's DMA was retired at the previous step's second barrier, or (the first
                    // step) it is retired here: everything but the 4 DMA loads just issued
                    if (ndb < d1) {
                        dma_stage(buf ^ (kN3BStageBufs - 1), ndb, nb);
                        asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
                    } else {
                        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
                    }
                }
                asm volatile("s_waitcnt lgkmcnt(0)\n\ts_barrier" ::: "memory");
            } else {
                if (q == kStage) {                  // stage J (by sub-tiles, twice over)
                    const int j = J * 64 + l;
                    const bool vj = j < N;
                    const double* p = tile_ptr(J) + l;
                    const double xj = vj ? p[0] : pad, yj = vj ? p[PS] : pad, zj = vj ? p[2 * PS] : pad;
                    const int li = n3b_lds(l);
                    sh.pj[buf][0][li] = xj; sh.pj[buf][0][li + 16] = xj;
                    sh.pj[buf][1][li] = yj; sh.pj[buf][1][li + 16] = yj;
                    sh.pj[buf][2][li] = zj; sh.pj[buf][2][li + 16] = zj;
                    if constexpr (FARF && MDQT_UFAR32) {   // relative to c_J = J's first ion (pj[.][0])
                        const float x32 = (float)(xj - uniform_f64(xj)), y32 = (float)(yj - uniform_f64(yj)),
                                    z32 = (float)(zj - uniform_f64(zj));
                        sh.pj32[0][li] = x32; sh.pj32[0][li + 16] = x32;
                        sh.pj32[1][li] = y32; sh.pj32[1][li + 16] = y32;
                        sh.pj32[2][li] = z32; sh.pj32[2][li + 16] = z32;
                    }
                    if (l < BW) {
                        if (plan) {                 // (P, db, b): one word per wave
                            sh.pw[buf][l] = plan[((size_t)(P - a.Plo) * a.nd + db) * (BW * BW) + b * BW + l];
                        } else {
                            int w = 2;              // class 0 (unsorted: every tile pair, per-pair image)
                            if (srt && P * BW + l < T) {
                                double g2;
                                int sm = 0;
                                w = n3b_pack_class(n3b_classify<VARIANT == 1>(a, c.invL, rad, P * BW + l, J, g2,
                                                                              AXP ? &sm : nullptr), sm);
                            }
                            sh.pw[buf][l] = make_uint2((unsigned)w, 0xFFu);
                        }
                    }
                }
#if !defined(MDQT_EXPT_NOBAR)                       // (diagnostic build: no J-step barriers, wrong results)
                __syncthreads();
#endif
            }
            const double (*pj)[128] = sh.pj[buf];
            const double* mj = sh.mjs[J == T - 1];
            const int tw = __builtin_amdgcn_readfirstlane((int)sh.pw[buf][q].x);
            const int cls = (tw & 15) - 2;
            const bool mine = vI && (db > 0 || J >= I);
            const bool diag = (db == 0 && J == I);
            // this wave's sub-tile groups, by pair form (k_n3b_plan)
            const unsigned word = __builtin_amdgcn_readfirstlane(sh.pw[buf][q].y);
            const unsigned groups = word & 15u;
            if (mine && cls >= 0 && groups) {
                // blocked i accumulation: the tile pair's steps into a fresh sum, those into the
                // block distance's sum, those into the run's (a run is ~1e5 pair terms at N = 1e6;
                // in spatial order they arrive in coherent groups, and one serial chain would
                // carry their rounding: momentum |sum F| / mean |F| 1.8e-8 -> 1e-10 at C4)
                double tx = 0., ty = 0., tz = 0.;
                n3b_tile_pair<VARIANT, GUARD, POT, AXP>(a, c, l, diag, ragN && (I == T - 1 || J == T - 1), tw, word, xi, yi,
                                                        zi, mi, pj, mj, sh.pj32, ax, ay, az, tx, ty, tz, cf32, invl32,
                                                        rc2f);
                bx += tx; by += ty; bz += tz;
            }
            if (kDbuf && plan && q == kStage) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");   // the DMA retired
#if !defined(MDQT_EXPT_NOBAR)
            __syncthreads();
#endif
            if (kDbuf && plan) buf ^= kN3BStageBufs - 1;
            if (q < (POT ? 1 : 3)) {                // j side of J's rows -> j-slot db
                const int l = lane_opaque(l0);
                const int li = n3b_lds(l);
                // the 16 waves' two copies, summed as a fixed pairwise tree (dependency depth 5,
                // not 16), then zeroed for the next J step
                double s16[BW];
#pragma unroll
                for (int w = 0; w < BW; ++w) {
                    s16[w] = sh.accj[w][q][li] + sh.accj[w][q][li + 16];
                    sh.accj[w][q][li] = 0.;
                    sh.accj[w][q][li + 16] = 0.;
                }
#pragma unroll
                for (int h = BW / 2; h >= 1; h /= 2)
#pragma unroll
                    for (int w = 0; w < h; ++w) s16[w] = s16[2 * w] + s16[2 * w + 1];
                a.slots[(size_t)db * plane + (size_t)q * a.Npad + J * 64 + l] = POT ? s16[0] : -s16[0];
            }
        }
        if (vI) {                                   // (0 + bx: the first block distance's partial as is)
            double* fi = fiptr();
            fi[0] = fi_first ? 0. + bx : fi[0] + bx;
            fi[FS] = fi_first ? 0. + by : fi[FS] + by;
            fi[2 * FS] = fi_first ? 0. + bz : fi[2 * FS] + bz;
        }
        fi_first = false;
    }
    if (vI) {                                       // i side -> i-slot nd + run
        double* fi = fiptr();
        double* o = a.slots + (size_t)(a.nd + run) * plane + I * 64 + lane_opaque(l0);
        const double r0 = fi_first ? 0. : fi[0], r1 = fi_first ? 0. : fi[FS], r2 = fi_first ? 0. : fi[2 * FS];
        if (MDQT_N3B_IRUN_LDS || fi_first) { o[0] = r0; o[a.Npad] = r1; o[2 * (size_t)a.Npad] = r2; }
    }
}


// k_pairs_n3b_pw's tile pairing of a block distance: wave k runs I tiles (bits 6k..6k+2, 6k+3..6k+5);
// without a plan the fixed pairing (k, 7 - k)
constexpr unsigned kN3BPairsDefault = (0u | 7u << 3) | (1u | 6u << 3) << 6 | (2u | 5u << 3) << 12 | (3u | 4u << 3) << 18;
static_assert(BW == 8, "the paired-wave pairing word holds 8 tiles");
// the 105 pairings of 8 tiles (pairing words as kN3BPairsDefault)
__constant__ const unsigned kN3BMatchings[105] = {0xfac688, 0xf74688, 0xd7c688, 0xfab888, 0xf73888, 0xd7b888, 0xfa3a88, 0xf33a88, 0xd3ba88, 0xf63c88, 0xf2bc88, 0xb3bc88, 0xd63e88, 0xd2be88, 0xb33e88, 0xfac650, 0xf74650, 0xd7c650, 0xfab850, 0xf73850, 0xd7b850, 0xfa3a50, 0xf33a50, 0xd3ba50, 0xf63c50, 0xf2bc50, 0xb3bc50, 0xd63e50, 0xd2be50, 0xb33e50, 0xfac458, 0xf74458, 0xd7c458, 0xfaa858, 0xf72858, 0xd7a858, 0xfa2a58, 0xf32a58, 0xd3aa58, 0xf62c58, 0xf2ac58, 0xb3ac58, 0xd62e58, 0xd2ae58, 0xb32e58, 0xfab460, 0xf73460, 0xd7b460, 0xfaa660, 0xf72660, 0xd7a660, 0xf9aa60, 0xef2a60, 0xcfaa60, 0xf5ac60, 0xeeac60, 0xafac60, 0xd5ae60, 0xceae60, 0xaf2e60, 0xfa3468, 0xf33468, 0xd3b468, 0xfa2668, 0xf32668, 0xd3a668, 0xf9a868, 0xef2868, 0xcfa868, 0xf1ac68, 0xee2c68, 0x8fac68, 0xd1ae68, 0xce2e68, 0x8f2e68, 0xf63470, 0xf2b470, 0xb3b470, 0xf62670, 0xf2a670, 0xb3a670, 0xf5a870, 0xeea870, 0xafa870, 0xf1aa70, 0xee2a70, 0x8faa70, 0xb1ae70, 0xae2e70, 0x8eae70, 0xd63478, 0xd2b478, 0xb33478, 0xd62678, 0xd2a678, 0xb32678, 0xd5a878, 0xcea878, 0xaf2878, 0xd1aa78, 0xce2a78, 0x8f2a78, 0xb1ac78, 0xae2c78, 0x8eac78};
// a sub-tile group's estimated VALU instructions per lane (16 steps; the pairing's weights per wave-step of
// each pair form — exact, mid, far, very far, ultra far, f32 ultra far — uniform image / per-pair image; the
// ragged tile's exact form)
#ifndef MDQT_N3B_PAIR_COST
#define MDQT_N3B_PAIR_COST 0
#endif
__device__ __forceinline__ unsigned n3b_pair_cost(int level, bool uni, bool rag) {
#if MDQT_N3B_PAIR_COST
    // (round 6 A/B) issue slots per step from the forms' instruction costs (profiles/r06f_ubench_forms.txt:
    // v_rsq_f64 ~3.3 slots, f32 transcendentals ~2.4, plain f32 0.5)
    constexpr unsigned wu[6] = {43u, 41u, 38u, 33u, 28u, 18u}, wi[6] = {50u, 47u, 44u, 38u, 31u, 31u};
#else
    constexpr unsigned wu[6] = {39u, 36u, 31u, 27u, 25u, 9u}, wi[6] = {48u, 44u, 38u, 32u, 32u, 32u};
#endif
    return 16u * (rag ? 52u : uni ? wu[level] : wi[level]);
}

// ------------------------------------------------------------------------------------------
// Paired waves (round 6, option force_n3b_pairs): the blocks, plan, slots and reduction of k_pairs_n3b
// with a workgroup of BW / 2 = 4 waves, each running TWO of block P's 8 I tiles against every J tile of
// the block distance — tiles paired per block distance by k_n3b_plan, the one with the most estimated
// work with the one with the least (n3b_pairing).  k_pairs_n3b's J-step barriers wait for the busiest of
// its 8 waves, and within a block distance the same tiles are the busy ones (the I tiles nearest block Q):
// the busiest wave of a J step carried 1.19-1.28 x the mean (k_n3b_census bal, tools/jstep_balance.py),
// a no-barrier timing build ran 4-12 % faster.  A wave's two tile pairs of a J step add to one j
// accumulator (the J tile is the same), and the combine sums 4 of them; the I positions of the wave's two
// tiles are loaded once per block distance, the run's i sums are per tile in LDS.  LDS 31 KB: five
// workgroups per CU.  Deterministic (the pairing is a function of the positions), not bit-identical to
// k_pairs_n3b (another summation tree on the j side).
// ------------------------------------------------------------------------------------------
constexpr int NWP = BW / 2;                         // waves per workgroup
template <int W>
struct N3BSharedPW {
    double pj[3][128];                              // J positions by sub-tiles twice over (n3b_lds)
    float pj32[3][128];                             // fl32(xj - c_J) (the f32 ultra-far form)
    double accj[W][3][128];                         // per-wave j accumulators
    double mjs[2][128];                             // J validity weights: all ones / the ragged last tile's
    double etab[64];                                // 2^(k/64) (MDQT_EXP_TAB)
    double irun[BW][3][64];                         // the run's i sums, per I tile of the block
    uint2 pw[BW];                                   // the J step's plan words, per I tile
};
#ifndef MDQT_N3B_PW_WPE
#define MDQT_N3B_PW_WPE 5                           // waves per SIMD: five 4-wave workgroups per CU (LDS 31 KB)
#endif
template <int VARIANT, bool GUARD, bool POT = false, bool AXP = false>
__global__ __launch_bounds__(NWP * 64) __attribute__((amdgpu_waves_per_eu(VARIANT == 1 ? MDQT_N3B_PW_WPE : 4, VARIANT == 1 ? MDQT_N3B_PW_WPE : 4)))
void k_pairs_n3b_pw(N3BArgs a) {
    __shared__ N3BSharedPW<NWP> sh;
    double* const etab = sh.etab;
    stage_exp_tab(etab);
    const int q = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), l = threadIdx.x & 63;   // q: wave-uniform
    const int l0 = l;
    const int nP = a.Phi - a.Plo;
    const int P = a.Plo + (MDQT_N3B_ORDER ? (int)blockIdx.x % nP : (int)blockIdx.x / a.R);
    const int run = MDQT_N3B_ORDER ? (int)blockIdx.x / nP : (int)blockIdx.x % a.R;
    const int d0 = run * a.runlen, d1 = min(a.nd, d0 + a.runlen);
    const PairC c = {a.L, a.micT, a.micGuard, a.Rcut, a.lDeb, a.invlDeb, 1. / a.L, a.rc2, etab};
    const int T = a.T, N = a.N, S = a.S;
    const bool ragN = (N & 63) != 0;
    const bool srt = a.use_sort != 0;
    const int PS = srt ? a.Npad : S;
    auto tile_ptr = [&](int tile) { return srt ? a.Rs + tile * 64 : tile_base(a.Rall, tile, S); };
    const double pad = (double)(l + 1) * 0x1p-10;  // pad ions: distinct points (pair_ft_cut: r > 0)
    constexpr bool FARF = VARIANT == 1 && !GUARD && VARIANT == 1 && MDQT_N3_CUT;
    const N3BRadii rad = n3b_radii<VARIANT, POT>(a);
    auto sgpr_f = [](float v) { return __int_as_float(__builtin_amdgcn_readfirstlane(__float_as_int(v))); };
    const float cf32 = sgpr_f((float)(a.invlDeb * kNegLog2e)), invl32 = sgpr_f((float)a.invlDeb),
                rc2f = sgpr_f((float)a.rc2);
    const uint2* plan = a.plan;
    constexpr int kStage = NWP - 1;                 // stages J; waves 0..2 combine the j sums
#pragma unroll
    for (int k = 0; k < 3; ++k) {
        sh.accj[q][k][l] = 0.; sh.accj[q][k][l + 64] = 0.;
        sh.irun[q][k][l] = 0.; sh.irun[q + NWP][k][l] = 0.;
    }
    double* ax = sh.accj[q][0];
    double* ay = sh.accj[q][1];
    double* az = sh.accj[q][2];
    if (q == kStage) {
        const int li = n3b_lds(l);
        const double m1 = (T - 1) * 64 + l < N ? 1. : 0.;
        sh.mjs[0][li] = 1.; sh.mjs[0][li + 16] = 1.;
        sh.mjs[1][li] = m1; sh.mjs[1][li + 16] = m1;
    }
    const size_t plane = (size_t)3 * a.Npad;
    const unsigned* jsteps = plan ? (const unsigned*)(plan + (size_t)(a.Phi - a.Plo) * a.nd * (BW * BW)) : nullptr;
    auto half_db = [&](int db) { return !(a.NB & 1) && db == a.NB / 2 && P >= a.NB / 2; };
    for (int db = d0; db < d1; ++db) {
        if (half_db(db)) continue;
        const int Q = (P + db) % a.NB;
        const size_t jw = 2 * ((size_t)(P - a.Plo) * a.nd + db);
        const unsigned jmask = jsteps ? __builtin_amdgcn_readfirstlane(jsteps[jw]) : ~0u;
        // the wave's two I tiles of this block distance (k_n3b_plan; without a plan: q and 7 - q)
        const unsigned pr = jsteps ? __builtin_amdgcn_readfirstlane(jsteps[jw + 1]) : kN3BPairsDefault;
        const int tA = (pr >> (6 * q)) & 7, tB = (pr >> (6 * q + 3)) & 7;
        const int IA = P * BW + tA, IB = P * BW + tB;
        const bool vA = IA < T, vB = IB < T;
        double xA = pad, yA = pad, zA = pad, mA = 0., xB = pad, yB = pad, zB = pad, mB = 0.;
        if (vA && IA * 64 + l < N) {
            const double* p = tile_ptr(IA) + l;
            xA = p[0]; yA = p[PS]; zA = p[2 * PS]; mA = 1.;
        }
        if (vB && IB * 64 + l < N) {
            const double* p = tile_ptr(IB) + l;
            xB = p[0]; yB = p[PS]; zB = p[2 * PS]; mB = 1.;
        }
        double bxA = 0., byA = 0., bzA = 0., bxB = 0., byB = 0., bzB = 0.;
        bool work = false;
        for (int b = 0; b < BW; ++b) {
            const int J = Q * BW + b;
            if (J >= T) break;
            if (jsteps && !((jmask >> b) & 1u)) {   // every tile pair of this J step skipped (wave-uniform)
                if (q < (POT ? 1 : 3) && !a.tmask)
                    a.slots[(size_t)db * plane + (size_t)q * a.Npad + J * 64 + lane_opaque(l0)] = POT ? 0. : -0.;
                continue;
            }
            work = true;
            if (q == kStage) {                      // stage J (by sub-tiles, twice over) and the step's plan words
                const int j = J * 64 + l;
                const bool vj = j < N;
                const double* p = tile_ptr(J) + l;
                const double xj = vj ? p[0] : pad, yj = vj ? p[PS] : pad, zj = vj ? p[2 * PS] : pad;
                const int li = n3b_lds(l);
                sh.pj[0][li] = xj; sh.pj[0][li + 16] = xj;
                sh.pj[1][li] = yj; sh.pj[1][li + 16] = yj;
                sh.pj[2][li] = zj; sh.pj[2][li + 16] = zj;
                if constexpr (FARF && MDQT_UFAR32) {
                    const float x32 = (float)(xj - uniform_f64(xj)), y32 = (float)(yj - uniform_f64(yj)),
                                z32 = (float)(zj - uniform_f64(zj));
                    sh.pj32[0][li] = x32; sh.pj32[0][li + 16] = x32;
                    sh.pj32[1][li] = y32; sh.pj32[1][li + 16] = y32;
                    sh.pj32[2][li] = z32; sh.pj32[2][li + 16] = z32;
                }
                if (l < BW) {
                    if (plan) {
                        sh.pw[l] = plan[((size_t)(P - a.Plo) * a.nd + db) * (BW * BW) + b * BW + l];
                    } else {
                        int w = 2;
                        if (srt && P * BW + l < T) {
                            double g2;
                            int sm = 0;
                            w = n3b_pack_class(n3b_classify<VARIANT == 1>(a, c.invL, rad, P * BW + l, J, g2,
                                                                          AXP ? &sm : nullptr), sm);
                        }
                        sh.pw[l] = make_uint2((unsigned)w, 0xFFu);
                    }
                }
            }
#if !defined(MDQT_EXPT_NOBAR)                       // (diagnostic build: no J-step barriers, wrong results)
            __syncthreads();
#endif
            const double (*pj)[128] = sh.pj;
            const double* mj = sh.mjs[J == T - 1];
#pragma unroll 1
            for (int u = 0; u < 2; ++u) {            // the wave's two tile pairs (I_A, J), (I_B, J)
                const int tI = u ? tB : tA;
                const int I = P * BW + tI;
                const int tw = __builtin_amdgcn_readfirstlane((int)sh.pw[tI].x);
                const unsigned word = __builtin_amdgcn_readfirstlane(sh.pw[tI].y);
                const bool mine = (u ? vB : vA) && (db > 0 || J >= I);
                if (mine && (tw & 15) >= 2 && (word & 15u)) {
                    double tx = 0., ty = 0., tz = 0.;
                    n3b_tile_pair<VARIANT, GUARD, POT, AXP>(a, c, l, db == 0 && J == I, ragN && (I == T - 1 || J == T - 1),
                                                            tw, word, u ? xB : xA, u ? yB : yA, u ? zB : zA,
                                                            u ? mB : mA, pj, mj, sh.pj32, ax, ay, az, tx, ty, tz, cf32,
                                                            invl32, rc2f);
                    if (u) { bxB += tx; byB += ty; bzB += tz; }
                    else { bxA += tx; byA += ty; bzA += tz; }
                }
            }
#if !defined(MDQT_EXPT_NOBAR)
            __syncthreads();
#endif
            if (q < (POT ? 1 : 3)) {                // j side of J's rows -> j-slot db: the 4 waves' two copies
                const int l = lane_opaque(l0);
                const int li = n3b_lds(l);
                double s4[NWP];
#pragma unroll
                for (int w = 0; w < NWP; ++w) {
                    s4[w] = sh.accj[w][q][li] + sh.accj[w][q][li + 16];
                    sh.accj[w][q][li] = 0.;
                    sh.accj[w][q][li + 16] = 0.;
                }
#pragma unroll
                for (int h = NWP / 2; h >= 1; h /= 2)
#pragma unroll
                    for (int w = 0; w < h; ++w) s4[w] = s4[2 * w] + s4[2 * w + 1];
                a.slots[(size_t)db * plane + (size_t)q * a.Npad + J * 64 + l] = POT ? s4[0] : -s4[0];
            }
        }
        if (work) {                                 // this block distance's i sums into the run's, per tile
            const int lo = lane_opaque(l0);
            double* fa = sh.irun[tA][0] + lo;
            fa[0] += bxA; fa[64] += byA; fa[128] += bzA;
            double* fb = sh.irun[tB][0] + lo;
            fb[0] += bxB; fb[64] += byB; fb[128] += bzB;
        }
    }
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 2; ++u) {                   // i side -> i-slot nd + run: tiles q and q + 4
        const int tI = q + u * NWP, I = P * BW + tI;
        if (I < T) {
            const int lo = lane_opaque(l0);
            const double* f = sh.irun[tI][0] + lo;
            double* o = a.slots + (size_t)(a.nd + run) * plane + I * 64 + lo;
            o[0] = f[0]; o[a.Npad] = f[64]; o[2 * (size_t)a.Npad] = f[128];
        }
    }
}

// force_tail_mode 1, after the call's per-sub-tile tail sums are complete (all-reduced over the
// ranks when sharded): every tile with a sub-tile sum that, with the sum's rounding (x (1 + 1e-12)),
// exceeds eps is listed for k_tail_fix (st[3] the list length; the same list on every rank); the
// other sums' largest goes into the running maximum st[0] — the bound every ion met after the fix —
// and the largest of all into st[1] (what the skip radius alone gave); st[2] counts the tiles over
// eps (the host widens r_t when it grows), st[4] the measured calls.  Positive doubles order as
// their bit patterns.
__global__ __launch_bounds__(256) void k_tail_max(const double* __restrict__ tailb, int T, double eps,
                                                  unsigned long long* st, int* list) {
    double m = 0., mr = 0.;
    unsigned long long nf = 0;
    for (int t = blockIdx.x * 256 + threadIdx.x; t < T; t += gridDim.x * 256) {
        const double v = fmax(fmax(tailb[4 * t], tailb[4 * t + 1]), fmax(tailb[4 * t + 2], tailb[4 * t + 3]));
        mr = fmax(mr, v);
        if (v * (1. + 1e-12) > eps) {
            ++nf;
            list[atomicAdd(st + 3, 1ull)] = t;
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

// force_tail_mode 1, enforcement: every listed tile's ions get their force recomputed exactly —
// all pairs inside L/2 (SpeedUp:213-224: per-pair minimum image, the exact cutoff, the fast pair
// form's values), over every J tile whose box is within L/2 of the tile's box — and the result
// REPLACES their rows of `out`: on the rank that owns the tile's block (F, or its dense partial
// before the reduce-scatter; the other ranks write 0 there, so the sum over the ranks is the exact
// force).  Replacing (not adding the dropped pairs) holds whatever the block kernel skipped: whole
// tile pairs, sub-tile groups, far forms.  One workgroup of 4 waves per listed tile (grid-stride
// over the list), wave q classifying the J tiles q*64 + l + 256 k lane-parallel and walking its
// ballot; the waves' sums combined in wave order: deterministic.  Each ion belongs to one tile, so
// `out` has one writer per ion.  With an empty list (the normal case) every workgroup reads st[3]
// and returns.
// POT (Epotential on the plan): the listed tiles' U_i = sum of u over every pair inside L/2 (pair_u<1>),
// component 0 of `out` (the per-ion potential rows)
template <bool POT = false>
__global__ __launch_bounds__(256) void k_tail_fix(N3BArgs a, const unsigned long long* __restrict__ st,
                                                  const int* __restrict__ list, double* __restrict__ out) {
    __shared__ double part[4][3][64];
    const int n = (int)st[3];
    const int q = threadIdx.x >> 6, l = threadIdx.x & 63;
    const PairC c = {a.L, a.micT, a.micGuard, a.Rcut, a.lDeb, a.invlDeb, 1. / a.L, a.rc2, nullptr};
    const double rcut2 = a.Rcut * a.Rcut;
    const N3BRadii none = {rcut2, INFINITY, INFINITY, INFINITY, INFINITY, INFINITY};
    const int T = a.T, N = a.N, PS = a.Npad;
    for (int k = blockIdx.x; k < n; k += gridDim.x) {
        const int I = __builtin_amdgcn_readfirstlane(list[k]);
        const bool own = I / BW >= a.Plo && I / BW < a.Phi;
        const int i = I * 64 + l;
        const bool vi = i < N;
        const double xi = vi ? a.Rs[i] : 0., yi = vi ? a.Rs[PS + i] : 0., zi = vi ? a.Rs[2 * PS + i] : 0.;
        // per J tile a 64-term partial, added with its rounding error kept (Neumaier): the exact
        // pass's sum is accurate to a few ulp of |F| rather than carrying ~1e5 rounded additions
        double fx = 0., fy = 0., fz = 0., ex = 0., ey = 0., ez = 0.;
        auto nadd = [](double& s, double& e, double v) {
            const double t = s + v;
            e += fabs(s) >= fabs(v) ? (s - t) + v : (v - t) + s;
            s = t;
        };
        for (int j0 = q * 64; own && j0 < T; j0 += 256) {
            const int Jl = j0 + l;
            bool in = false;
            if (Jl < T) {
                double g2;
                (void)n3b_classify<false>(a, c.invL, none, I, Jl, g2);
                in = g2 < rcut2;
            }
            unsigned long long m = __ballot(in);
            while (m) {
                const int J = j0 + __builtin_ctzll(m);
                m &= m - 1;
                const int j = J * 64 + l;
                const int nj = min(64, N - J * 64);
                const double xl = j < N ? a.Rs[j] : 0., yl = j < N ? a.Rs[PS + j] : 0., zl = j < N ? a.Rs[2 * PS + j] : 0.;
                double px = 0., py = 0., pz = 0.;
                for (int t = 0; t < nj; ++t) {
                    auto lane_t = [t](double v) {
                        return __hiloint2double(__builtin_amdgcn_readlane(__double2hiint(v), t),
                                                __builtin_amdgcn_readlane(__double2loint(v), t));
                    };
                    double dx = xi - lane_t(xl), dy = yi - lane_t(yl), dz = zi - lane_t(zl);
                    mic_r(dx, dy, dz, c);
                    if constexpr (POT) {
                        px += pair_u<1>(dx, dy, dz, c);            // 0 beyond L/2 and for i = j
                    } else {
                        const double ft = pair_ft<1>(dx, dy, dz, c);   // 0 beyond L/2 and for i = j
                        px = fma(dx, ft, px); py = fma(dy, ft, py); pz = fma(dz, ft, pz);
                    }
                }
                nadd(fx, ex, px); nadd(fy, ey, py); nadd(fz, ez, pz);
            }
        }
        part[q][0][l] = fx + ex; part[q][1][l] = fy + ey; part[q][2][l] = fz + ez;
        __syncthreads();
        if (q == 0 && vi) {
            const int ion = a.perm[i];
            const int w = ion / a.S;
            double* o = out + (size_t)w * 3 * a.S + (ion - w * a.S);
#pragma unroll
            for (int c3 = 0; c3 < (POT ? 1 : 3); ++c3)
                o[(size_t)c3 * a.S] = ((part[0][c3][l] + part[1][c3][l]) + part[2][c3][l]) + part[3][c3][l];
        }
        __syncthreads();
    }
}

// the AXP instance where tile pairs whose image varies on one axis can be evaluated: their pairs are >=
// L/2 - (the two tiles' extents) apart on that axis, so only when the skip radius reaches within two tile
// widths (L (64/N)^(1/3)) of L/2 (C3, C5: r_s = L/2; not N = 1M, r_s = 61 < 80.6 - 12.9).  A function of
// the call's parameters alone: every rank of a sharded run, and every call of one configuration, takes
// the same kernel.
__host__ __device__ static bool n3b_axp(const N3BArgs& a) {
    return a.ax1 && a.use_sort != 0 && a.Rskip > 0.5 * a.L - 2. * a.L * cbrt(64. / a.N);
}

// Census of the block kernel's work (diagnostic; bench.py's large lines): k_pairs_n3b's loop over
// this rank's block pairs without the pair terms — every tile pair classified by n3b_classify and
// its sub-tile groups by the same sub-block gaps, counted by the path the kernel takes, as
// lane-steps (its work: 64 per step of a wave, 16 steps per sub-tile group; 40 steps on a diagonal
// tile) in out[0, kCensus) and as distinct ion pairs in out[kCensus, 2 kCensus).  Classes:
// 0 skipped (boxes beyond L/2), 1 skipped by the tail radius, 2 ragged last tile (exact, per-pair
// image), 3 exact per-pair image, 4 exact uniform image, 5 far per-pair, 6 far uniform, 7 very far
// per-pair (ultra far with a per-pair image included), 8 very far uniform, 9 ultra far uniform (f64),
// 10 ultra far uniform in f32, 11 skipped sub-tile groups of evaluated tile pairs, 12 mid per-pair,
// 13 mid uniform (round 4: appended, the earlier indices kept), 14 ultra far with a one-axis per-pair image
// (round 6: the f64 ultra-far form on the AXP path).  One workgroup
// per (block P, block distance db); thread (b, q) takes tile pair (16 P + q, 16 Q + b) as the
// kernel's wave q at J-step b does.
// bw (optional): the evaluated lane-steps (every class but the skipped ones) per block of this rank,
// bw[P - Plo] — the work each block's workgroups do, for the ranks' load balance (mdqt_force_block_work)
// bal (optional, round 6): the J steps' balance over the workgroup's 8 waves — each tile pair's VALU
// instructions estimated from its groups' classes (kCensusValu: per wave-step of each form, from the ISA
// counts in docs/FORCES.md) — bal[0] += sum over the waves, bal[1] += the busiest wave's, bal[2] += 1 per
// J step with work: bal[1] / (bal[0] / 8) is the barrier-bound excess of the lock-step J loop
__constant__ const unsigned kCensusValu[kCensus] = {0, 0, 52, 48, 39, 38, 31, 32, 27, 25, 9, 0, 44, 36, 28};
__global__ __launch_bounds__(256) void k_n3b_census(N3BArgs a, unsigned long long* __restrict__ out,
                                                    unsigned long long* __restrict__ bw,
                                                    unsigned long long* __restrict__ bal) {
    __shared__ unsigned long long h[2 * kCensus];
    __shared__ unsigned long long hb;
    const int t = threadIdx.x;
    if (t < 2 * kCensus) h[t] = 0;
    if (t == 0) hb = 0;
    __syncthreads();
    unsigned long long cost = 0;                    // this tile pair's estimated VALU (bal)
    auto add = [&](int k, unsigned long long steps, unsigned long long pairs) {
        atomicAdd(&h[k], steps);
        atomicAdd(&h[kCensus + k], pairs);
        if (k != 0 && k != 1 && k != 11) atomicAdd(&hb, steps);
        cost += (steps / 64) * kCensusValu[k];
    };
    const int P = a.Plo + (int)blockIdx.x / a.nd, db = (int)blockIdx.x % a.nd;
    const int q = t & (BW - 1), b = t / BW;
    const int Q = (P + db) % a.NB;
    const int I = P * BW + q, J = Q * BW + b;
    const bool half = !(a.NB & 1) && db == a.NB / 2 && P >= a.NB / 2;   // the other half covers it
    if (!half && I < a.T && J < a.T && (db > 0 || J >= I)) {
        const N3BRadii rad = n3b_radii<1, false>(a);
        double g2;
        int sm = 0;
        const double4 t4 = n3b_classify<true>(a, 1. / a.L, rad, I, J, g2, &sm);
        const bool diag = db == 0 && J == I;
        // (a per-pair image on one axis, AXP instance: levels 4 and 5 in the f64 ultra-far form, class 14)
        constexpr bool AX1U = MDQT_N3B_AX1 != 0 && (MDQT_N3B_AX1_LEVELS & 16u) != 0;
        const bool ax1p = AX1U && n3b_axp(a) && ((n3b_pack_class(t4, sm) >> 28) & 3);
        const double nI = (double)min(64, a.N - I * 64), nJ = (double)min(64, a.N - J * 64);
        const bool rag = (a.N & 63) && (I == a.T - 1 || J == a.T - 1);
        const bool uni = ((int)t4.w & 1) != 0;
        // the class of a group at far level gl (the kernel's dispatch)
        auto cls_of = [&](unsigned gl) {
            if (rag) return 2;
            if (uni) return gl == 5 ? 10 : gl == 4 ? 9 : gl == 3 ? 8 : gl == 2 ? 6 : gl == 1 ? 13 : 4;
            return (ax1p && gl >= 4) ? 14 : gl >= 3 ? 7 : gl == 2 ? 5 : gl == 1 ? 12 : 3;
        };
        if (t4.w < 0.) {
            add(t4.w == -2. ? 1 : 0, 4096ull, (unsigned long long)(nI * nJ));
        } else if (diag) {
            add(cls_of(0), 2560ull, (unsigned long long)(nI * (nI - 1) / 2));
        } else {
            const int T4 = 4 * a.T;
            const double hj2 = raw_half2(a.boxes, a.T, J);
            unsigned act = 0, mm = 0, mf = 0, mv = 0, mu = 0, m32 = 0;
            double np[4] = {0., 0., 0., 0.};       // ion pairs per group
            for (int sa = 0; sa < 4; ++sa)
                for (int sb = 0; sb < 4; ++sb) {
                    const double sg = sub_gap2(a.subboxes, T4, 4 * I + sa, 4 * J + sb, a.L, 1. / a.L);
                    const unsigned bit = 1u << (4 * sa + sb);
                    if (sg <= rad.rc2) act |= bit;
                    if (sg > rad.rm2) mm |= bit;
                    if (sg > rad.rf2) mf |= bit;
                    if (sg > rad.rv2) mv |= bit;
                    if (sg > rad.ru2) mu |= bit;
                    if (sg > rad.ru32 && sg > 4. * hj2 &&   // (k_n3b_plan's level 5)
                        (!a.formm || !uni || sub_far2(a.subboxes, T4, 4 * I + sa, 4 * J + sb, a.L, 1. / a.L) < a.u32lim2))
                        m32 |= bit;
                    np[(sb - sa) & 3] += sub_count(a.N, 4 * I + sa) * sub_count(a.N, 4 * J + sb);
                }
            const unsigned g = a.use_sort == 1 ? sub_groups_of(act) : 0xFu;   // (2: nothing skipped)
            const unsigned lv = sub_group_levels(mm, mf, mv, mu, m32);
            for (int d = 0; d < 4; ++d)
                add((g >> d) & 1u ? cls_of((lv >> (4 * d)) & 15u) : 11, 1024ull, (unsigned long long)np[d]);
        }
    }
    if (bal) {                                      // the 8 threads of J step b: lanes 8 (b mod 8) .. + 7
        unsigned long long sm = cost, mx = cost;
#pragma unroll
        for (int off = 1; off < BW; off <<= 1) {
            sm += __shfl_xor(sm, off);
            const unsigned long long o = __shfl_xor(mx, off);
            mx = o > mx ? o : mx;
        }
        if (q == 0 && sm) {
            atomicAdd(bal, sm);
            atomicAdd(bal + 1, mx);
            atomicAdd(bal + 2, 1ull);
        }
        // schedules that move no work between waves (what a J-order change could reach): bal[3] the pairs
        // of J steps (b, b + 1) each run as two sub-steps with every wave on one of the two J tiles, the
        // best of the 256 choices; bal[4] the same pairs in lock-step; bal[5] per (P, db) the busiest
        // wave's sum over its 8 J steps (any J order's floor)
        const int lane = t & 63, base = lane & ~15;     // the pair's 16 costs: lanes base .. base + 15
        unsigned long long c16[16];
#pragma unroll
        for (int k = 0; k < 16; ++k) c16[k] = __shfl(cost, base + k);
        if (lane == base) {
            unsigned long long cur = 0, m0 = 0, m1 = 0, best = ~0ull;
            for (int k = 0; k < 8; ++k) { m0 = c16[k] > m0 ? c16[k] : m0; m1 = c16[8 + k] > m1 ? c16[8 + k] : m1; }
            cur = m0 + m1;
            for (unsigned S = 0; S < 256; ++S) {        // wave k in S: J step b first, b + 1 second
                unsigned long long a1 = 0, a2 = 0;
                for (int k = 0; k < 8; ++k) {
                    const unsigned long long x = c16[k], y = c16[8 + k];
                    const bool in = (S >> k) & 1u;
                    const unsigned long long f = in ? x : y, g = in ? y : x;
                    a1 = f > a1 ? f : a1;
                    a2 = g > a2 ? g : a2;
                }
                best = a1 + a2 < best ? a1 + a2 : best;
            }
            if (cur) { atomicAdd(bal + 3, best); atomicAdd(bal + 4, cur); }
        }
        unsigned long long rw = cost;                   // wave q's sum over the workgroup's 8 J steps
#pragma unroll
        for (int off = BW; off < 64; off <<= 1) rw += __shfl_xor(rw, off);
        __shared__ unsigned long long rws[BW];
        if (lane < BW) rws[lane] = 0;
        __syncthreads();
        if (lane < BW) atomicAdd(&rws[lane], rw);
        __syncthreads();
        if (t == 0) {
            unsigned long long m = 0;
            for (int k = 0; k < BW; ++k) m = rws[k] > m ? rws[k] : m;
            if (m) atomicAdd(bal + 5, m);
        }
        // 4 waves, each on two I tiles per J step (the pair's costs add): bal[6] the pairing of the heaviest
        // row with the lightest (per (P, db)), bal[7] the fixed pairing (q, 7 - q), bal[8] (q, q + 4) — each
        // the sum over J steps of 2 x the busiest wave's pair, comparable with bal[1]
        unsigned long long c64[BW * BW];
#pragma unroll
        for (int k = 0; k < BW * BW; ++k) c64[k] = __shfl(cost, k);   // c64[q + 8 b]
        if (t == 0) {
            unsigned long long row[BW];
            int ord[BW];
            for (int k = 0; k < BW; ++k) { row[k] = 0; ord[k] = k; }
            for (int b = 0; b < BW; ++b)
                for (int k = 0; k < BW; ++k) row[k] += c64[k + BW * b];
            for (int i = 1; i < BW; ++i)                // rows by cost, descending
                for (int j = i; j > 0 && row[ord[j]] > row[ord[j - 1]]; --j) { const int x = ord[j]; ord[j] = ord[j - 1]; ord[j - 1] = x; }
            unsigned long long hl = 0, fx = 0, f4 = 0, ps = 0;
            for (int b = 0; b < BW; ++b) {
                unsigned long long m1 = 0, m2 = 0, m3 = 0, m4 = 0;
                int os[BW];                             // this J step's own heavy-light pairing (bal[9])
                for (int k = 0; k < BW; ++k) os[k] = k;
                for (int i = 1; i < BW; ++i)
                    for (int j = i; j > 0 && c64[os[j] + BW * b] > c64[os[j - 1] + BW * b]; --j) { const int x = os[j]; os[j] = os[j - 1]; os[j - 1] = x; }
                for (int k = 0; k < BW / 2; ++k) {
                    const unsigned long long p4 = c64[os[k] + BW * b] + c64[os[BW - 1 - k] + BW * b];
                    m4 = p4 > m4 ? p4 : m4;
                }
                ps += m4;
                for (int k = 0; k < BW / 2; ++k) {
                    const unsigned long long p1 = c64[ord[k] + BW * b] + c64[ord[BW - 1 - k] + BW * b];
                    const unsigned long long p2 = c64[k + BW * b] + c64[BW - 1 - k + BW * b];
                    const unsigned long long p3 = c64[k + BW * b] + c64[k + BW / 2 + BW * b];
                    m1 = p1 > m1 ? p1 : m1; m2 = p2 > m2 ? p2 : m2; m3 = p3 > m3 ? p3 : m3;
                }
                hl += m1; fx += m2; f4 += m3;
            }
            unsigned long long bm = ~0ull;          // the best of the 105 pairings of this (P, db) (bal[10])
            for (int m = 0; m < 105; ++m) {
                const unsigned pw = kN3BMatchings[m];
                unsigned long long cm = 0;
                for (int b = 0; b < BW; ++b) {
                    unsigned long long mx = 0;
                    for (int k = 0; k < BW / 2; ++k) {
                        const unsigned long long v = c64[((pw >> (6 * k)) & 7) + BW * b] + c64[((pw >> (6 * k + 3)) & 7) + BW * b];
                        mx = v > mx ? v : mx;
                    }
                    cm += mx;
                }
                bm = cm < bm ? cm : bm;
            }
            if (hl) { atomicAdd(bal + 6, hl); atomicAdd(bal + 7, fx); atomicAdd(bal + 8, f4); atomicAdd(bal + 9, ps); atomicAdd(bal + 10, bm); }
        }
    }
    __syncthreads();
    if (t < 2 * kCensus && h[t]) atomicAdd(out + t, h[t]);
    if (bw && t == 0 && hb) atomicAdd(bw + (P - a.Plo), hb);
}

// The block kernel's plan (force calls in spatial order): every tile pair of this rank's block pairs
// classified once per call, before k_pairs_n3b, so that its staging lanes read one 8-byte word per
// tile pair instead of classifying — work the block kernel's other 15 waves waited out at every J
// step's barrier (the sub-tile classification there cost C5 +8 %).  plan[((P - Plo) nd
// + db) 256 + 16 b + q] is tile pair (16 P + q, 16 Q + b), Q = P + db mod NB: .x its class and
// uniform-image multiples (n3b_pack_class), .y its sub-tile groups by pair form:
//  * group d = the sub-blocks (a, (a + d) & 3) of the tile pair's 4 x 4 (16-ion sub-tiles; the block
//    kernel's lane 16 a + m runs them as its d-th 16-step group); its gap is the least of their four
//    sub-box gaps.  It runs iff that gap is within the skip radius (force_sort 1; 2 runs all), in the
//    pair form the gap allows (the far level every pair of the group reaches: each form's error
//    bound needs every pair that far apart, which the sub-boxes guarantee).  .y = groups | (the
//    groups of far level x) << (4 + 4 x), x = 0..4; 0xFF (all groups, exact form) where unused.
//  * tail sums (force_tail_mode 1, a.tailb): every pair the call drops inside L/2 — in a tile pair
//    the tail radius skips (class -2) or in a skipped group — is at least its sub-block gap apart, so
//    each ion of I sub-tile a loses at most sum_b n_b g(gap_ab) and each ion of J sub-tile b at most
//    sum_a n_a g(gap_ab); counted once per unordered tile pair, summed per sub-tile in LDS over the
//    workgroup and added to tailb (128 atomics per workgroup).
// One workgroup per (P, db), thread (b, q) — the census's decomposition.
// the plan kernel's occupancy (round 6, A/B r06p_plan_ab.txt, bit-identical): 3 waves per SIMD (168 VGPRs,
// 2 spilled) with the LDS boxes: plan stage N = 1M 9.4 -> 7.8 ms, C5 0.75 -> 0.58 ms; 4 (128 VGPRs, 37
// spilled) is slower than 2
#ifndef MDQT_PLAN_WPE
#define MDQT_PLAN_WPE 3
#endif
#ifndef MDQT_PLAN_LDS
#define MDQT_PLAN_LDS 1
#endif
#ifndef MDQT_EXPT_PLAN
#define MDQT_EXPT_PLAN 0                            // diagnostic builds only (wrong plans): bit 0 no tail terms, 1 no pairing sort,
                                                    // 2 no sub-tile work
#endif
template <int VARIANT, bool GUARD>
__global__ __launch_bounds__(256) __attribute__((amdgpu_waves_per_eu(MDQT_PLAN_WPE)))
void k_n3b_plan(N3BArgs a, uint2* __restrict__ plan) {
    __shared__ double ti[BW][4], tj[BW][4];
    __shared__ unsigned jm;
    constexpr bool FARF = VARIANT == 1 && !GUARD && MDQT_N3_CUT;
    const int t = threadIdx.x, q = t & (BW - 1), b = t / BW;
    const int Pl = (int)blockIdx.x / a.nd, db = (int)blockIdx.x % a.nd;
    const int P = a.Plo + Pl, Q = (P + db) % a.NB;
    const int I = P * BW + q, J = Q * BW + b;
    const bool tmeas = a.tailb != nullptr;
    if (tmeas && t < 4 * BW) { ti[t >> 2][t & 3] = 0.; tj[t >> 2][t & 3] = 0.; }
    if (t == 0) jm = 0u;
    // the workgroup's boxes in LDS (MDQT_PLAN_LDS): the BW I tiles' and BW J tiles' [12] box columns and
    // their 4 BW sub-tiles' [6] — each read once, coalesced, instead of per tile pair from L2 (the kernel's
    // ~190 global loads held ~200 VGPRs: 2 waves per SIMD); the same values, the same operations
    __shared__ double bI[12][BW], bJ[12][BW], sI[6][4 * BW], sJ[6][4 * BW];
    if constexpr (MDQT_PLAN_LDS) {
        const int T4 = 4 * a.T;
        for (int k = t; k < 12 * BW; k += BW * BW) {
            const int row = k / BW, c = k % BW;
            bI[row][c] = P * BW + c < a.T ? a.boxes[(size_t)row * a.T + P * BW + c] : 0.;
            bJ[row][c] = Q * BW + c < a.T ? a.boxes[(size_t)row * a.T + Q * BW + c] : 0.;
        }
        if (a.subboxes)
            for (int k = t; k < 6 * 4 * BW; k += BW * BW) {
                const int row = k / (4 * BW), c = k % (4 * BW);
                sI[row][c] = 4 * P * BW + c < T4 ? a.subboxes[(size_t)row * T4 + 4 * P * BW + c] : 0.;
                sJ[row][c] = 4 * Q * BW + c < T4 ? a.subboxes[(size_t)row * T4 + 4 * Q * BW + c] : 0.;
            }
    }
    __syncthreads();
    // box column accessors: LDS (row stride BW / 4 BW) or global ([12][T] / [6][4T])
    const double* const Bi = MDQT_PLAN_LDS ? &bI[0][q] : a.boxes + I;
    const double* const Bj = MDQT_PLAN_LDS ? &bJ[0][b] : a.boxes + J;
    const int bld = MDQT_PLAN_LDS ? BW : a.T;
    auto SBi = [&](int sa) -> const double* { return MDQT_PLAN_LDS ? &sI[0][4 * q + sa] : a.subboxes + 4 * I + sa; };
    auto SBj = [&](int sb) -> const double* { return MDQT_PLAN_LDS ? &sJ[0][4 * b + sb] : a.subboxes + 4 * J + sb; };
    const int sld = MDQT_PLAN_LDS ? 4 * BW : 4 * a.T;
    uint2 w = make_uint2(1u, 0xFFu);                // class -1 where the block kernel never looks
    double gi[4] = {0., 0., 0., 0.}, gj[4] = {0., 0., 0., 0.};   // this tile pair's tail terms per sub-tile
    const bool half = !(a.NB & 1) && db == a.NB / 2 && P >= a.NB / 2;
    // the paired-wave kernel's work estimate of this tile pair (n3b_pair_cost: from the geometry alone, the
    // same with force_sort 1 and 2, so that both take the same pairing and stay bit-identical)
    unsigned cest = 0;
    if (!half && I < a.T && J < a.T && (db > 0 || J >= I)) {
        const N3BRadii rad = n3b_radii<VARIANT, false>(a);
        const double invL = 1. / a.L;
        double g2;
        int sm;
        const int pw = n3b_pack_class(n3b_classify_p<VARIANT == 1>(Bi, Bj, bld, a.L, invL, a.Rcut, a.use_sort, rad, g2, &sm),
                                       VARIANT == 1 ? sm : 0);
        const int cls = (pw & 15) - 2;
        w.x = (unsigned)pw;
        const bool rag = (a.N & 63) && (I == a.T - 1 || J == a.T - 1);
        const bool uni = cls >= 0 && (cls & 1);
        if (db == 0 && J == I && !(g2 > rad.rc2)) cest = (rag ? 52u : uni ? 39u : 48u) * 40u;
        if ((db > 0 || J > I) && (cls >= 0 || (tmeas && cls == -2)) && !(MDQT_EXPT_PLAN & 4)) {   // (bit 2: timing only)
            double sg[4][4];
#pragma unroll
            for (int sa = 0; sa < 4; ++sa)
#pragma unroll
                for (int sb = 0; sb < 4; ++sb) sg[sa][sb] = sub_gap2_p(SBi(sa), SBj(sb), sld, a.L, invL);
            unsigned groups = 0u, lvm = 0u;
            double gm[4];
#pragma unroll
            for (int d = 0; d < 4; ++d)
                gm[d] = fmin(fmin(sg[0][d & 3], sg[1][(1 + d) & 3]), fmin(sg[2][(2 + d) & 3], sg[3][(3 + d) & 3]));
            // the f32 level needs J's raw box diagonal within the group's gap (kUfar32A/B): J's extents
            // read only where a group is that far
            const double gmax = fmax(fmax(gm[0], gm[1]), fmax(gm[2], gm[3]));
            const double hj4 = FARF && gmax > rad.ru32 ? 4. * raw_half2_p(Bj, bld) : 0.;
            int xs[4];                              // the groups' levels (the measured form bound)
            // (formm) the whole tile pair within u32lim2 under its image — tile boxes: every sub-block is
            bool tile_in = false;
            if (FARF && a.formm && gmax > rad.ru32 && uni)
                tile_in = sub_far2_p(Bi, Bj, bld, a.L, invL) < a.u32lim2;   // ([12][T]: centers, half extents first)
#pragma unroll
            for (int d = 0; d < 4; ++d) {
                int x = !FARF ? 0 : n3b_level(gm[d], rad);
                if (x == 5 && !(gm[d] > hj4)) x = 4;
                if (x == 5 && a.formm && uni && !tile_in) {   // f32 only where no pair can reach the cutoff (u32lim2)
                    double f2 = 0.;
#pragma unroll
                    for (int sa = 0; sa < 4; ++sa)
                        f2 = fmax(f2, sub_far2_p(SBi(sa), SBj((sa + d) & 3), sld, a.L, invL));
                    if (!(f2 < a.u32lim2)) x = 4;
                }
                xs[d] = x;
                if (gm[d] <= rad.rc2 && !(g2 > rad.rc2)) cest += n3b_pair_cost(x, uni, rag);
                if (a.use_sort != 1 || gm[d] <= rad.rc2) {
                    groups |= 1u << d;
                    lvm |= 1u << (4 * x + d);
                }
            }
            if (cls >= 0) w.y = groups | (lvm << 4);
            if (tmeas && !(MDQT_EXPT_PLAN & 1)) {        // (EXPT_PLAN bit 0: timing only)
                const double rcut2 = a.Rcut * a.Rcut;
                const float invl = (float)a.invlDeb, cf = (float)(a.invlDeb * kNegLog2e);
                constexpr bool AX1U = FARF && MDQT_N3B_AX1 != 0 && (MDQT_N3B_AX1_LEVELS & 16u) != 0;
                const bool ax1p = AX1U && n3b_axp(a) && ((pw >> 28) & 3);
#pragma unroll
                for (int sa = 0; sa < 4; ++sa)
#pragma unroll
                    for (int sb = 0; sb < 4; ++sb) {
                        const int d = (sb - sa) & 3;
                        const bool drop = cls == -2 || !((groups >> d) & 1u);
                        // the form the block kernel takes for the group (n3b_tile_pair): exact on a ragged
                        // tile pair; with a per-pair image levels >= 3 in the very-far form, but levels 4
                        // and 5 in the f64 ultra-far form on the one-axis path (AXP instance, LV bit 4)
                        const int e = (drop || !a.formm || rag) ? 0 : uni ? xs[d]
                                    : (ax1p && xs[d] >= 4) ? 4 : min(xs[d], 3);
                        if ((drop || e > 0) && sg[sa][sb] < rcut2) {
                            const double gd = drop ? tail_g(sg[sa][sb], invl, cf) : form_term(sg[sa][sb], invl, cf, e);
                            gi[sa] += sub_count(a.N, 4 * J + sb) * gd;
                            gj[sb] += sub_count(a.N, 4 * I + sa) * gd;
                        }
                    }
            }
        }
    }
    plan[((size_t)Pl * a.nd + db) * (BW * BW) + t] = w;
    if (tmeas) {
        // the workgroup's sums per sub-tile: I sub-tiles over b (lanes q, q + 16, q + 32, q + 48 of
        // each wave, then one LDS add per wave), J sub-tiles over q (16 consecutive lanes: b's own)
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            double vi = gi[u], vj = gj[u];
#pragma unroll
            for (int off = BW; off < 64; off <<= 1) vi += __shfl_xor(vi, off);
#pragma unroll
            for (int off = BW / 2; off >= 1; off >>= 1) vj += __shfl_xor(vj, off);
            if ((t & 63) < BW && vi > 0.) atomicAdd(&ti[q][u], vi);
            if (q == 0) tj[b][u] = vj;              // (one writer per b)
        }
    }
    // the J-step mask of (P, db): J step b has work iff one of its tile pairs has a class >= 0
    // (threads BW b .. BW b + BW - 1 are lanes BW (b mod 64/BW) .. of wave b / (64/BW))
    const unsigned long long wk = __ballot((int)(w.x & 15u) >= 2);
    if ((t & 63) == 0) {
        constexpr int per = 64 / BW;
        unsigned mw = 0u;
#pragma unroll
        for (int k = 0; k < per; ++k) mw |= ((wk >> (BW * k)) & ((1ull << BW) - 1)) ? 1u << k : 0u;
        atomicOr(&jm, mw << (per * (t >> 6)));
    }
    // k_pairs_n3b_pw's pairing (.y of the J-step word): the tiles' estimated work over the 8 J steps (threads
    // q, q + 8, ... hold tile q's tile pairs), the busiest tile with the least busy, and so on
    unsigned rc = cest;
#pragma unroll
    for (int off = BW; off < 64; off <<= 1) rc += __shfl_xor(rc, off);
    // lanes 0 .. BW-1 hold the BW tiles' sums (lane t: tile t mod BW); each of them takes its tile's place in
    // the order (descending by work, ties by tile: the stable insertion sort's order) and its field of the
    // pairing word — the busiest tile with the least busy, and so on, 6 bits per pair — OR-ed over the lanes
    // (round 6: one thread's serial sort cost the plan stage ~1.5 ms of 8 at N = 1M)
    unsigned pr = 0;
    {
        unsigned row[BW];
#pragma unroll
        for (int k = 0; k < BW; ++k) row[k] = __shfl(rc, k);
        int rk = 0;
#pragma unroll
        for (int k = 0; k < BW; ++k) rk += (row[k] > rc || (row[k] == rc && k < t)) ? 1 : 0;
        if (t < BW) pr = rk < BW / 2 ? (unsigned)t << (6 * rk) : (unsigned)t << (3 + 6 * (BW - 1 - rk));
#pragma unroll
        for (int off = 1; off < BW; off <<= 1) pr |= __shfl_xor(pr, off);
    }
    __syncthreads();
    if (t == 0 && !(MDQT_EXPT_PLAN & 2))          // (EXPT_PLAN bit 1: timing only)
        plan[(size_t)(a.Phi - a.Plo) * a.nd * (BW * BW) + (size_t)Pl * a.nd + db] = make_uint2(jm, pr);
    // the reduction's per-J-tile masks: J step b has work -> the block kernel writes J's j-slot db
    if (a.tmask && t < BW && ((jm >> t) & 1u))
        atomicOr(a.tmask + (size_t)(Q * BW + t) * a.tmw + (db >> 6), 1ull << (db & 63));
    if (tmeas) {
        if (t < 4 * BW) {
            const int k = t >> 2, u = t & 3;
            if (ti[k][u] > 0.) atomicAdd(a.tailb + 4 * (P * BW + k) + u, ti[k][u]);
            if (tj[k][u] > 0.) atomicAdd(a.tailb + 4 * (Q * BW + k) + u, tj[k][u]);
        }
    }
}

// canonical per-ion sum of the slots this rank wrote: j-slots db = 0 .. nd-1, then i-slots.
// out: world 1 -> F [3][S]; sharded -> the rank's dense partial [world][3][S] (reduce-scattered)
// With the plan's per-J-tile masks (a.tmask) only the j-slots the block kernel wrote are read — the
// others held the -0 of empty J steps, and acc + -0 = acc: the same sum, bit for bit, without ~2/3 of
// the reads at N = 1M.  The masks are wave-uniform (a wave is one J tile): 8 slot loads in flight per
// round, added in ascending db order.
__global__ __launch_bounds__(256) void k_n3b_reduce(N3BArgs a, double* __restrict__ out) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    const int k = blockIdx.y;
    if (g >= a.N) return;
    const int B = (g >> 6) / BW;
    const size_t plane = (size_t)3 * a.Npad;
    const double* p = a.slots + (size_t)k * a.Npad + g;
    double acc = 0.;
    if (a.tmask) {
        const unsigned long long* tm = a.tmask + (size_t)(g >> 6) * a.tmw;
        for (int w = 0; w < a.tmw; ++w) {
            // (readfirstlane returns int: each half zero-extended, not sign-extended)
            unsigned long long m = (unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)tm[w]) |
                                   ((unsigned long long)(unsigned)__builtin_amdgcn_readfirstlane((unsigned)(tm[w] >> 32)) << 32);
            while (m) {
                int idx[8];
                int n = 0;
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (m) { idx[u] = 64 * w + __builtin_ctzll(m); m &= m - 1; n = u + 1; }
                double v[8];
#pragma unroll
                for (int u = 0; u < 8; ++u) v[u] = u < n ? p[(size_t)idx[u] * plane] : 0.;
#pragma unroll
                for (int u = 0; u < 8; ++u)
                    if (u < n) acc = acc + v[u];
            }
        }
    } else {
        for (int db = 0; db < a.nd; ++db) {
            const int P = (B - db + a.NB) % a.NB;
            const bool skip = !(a.NB & 1) && db == a.NB / 2 && P >= a.NB / 2;
            if (!skip && P >= a.Plo && P < a.Phi) acc = acc + p[(size_t)db * plane];
        }
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

// the plan (k_n3b_plan) of a force or potential call in spatial order, its per-J-tile masks zeroed first
static hipError_t launch_n3b_plan(const N3BArgs& a, int variant, hipStream_t s) {
    const int nplan = (a.Phi - a.Plo) * a.nd;
    if (a.plan && nplan > 0) {
        if (!a.use_sort || !a.boxes || !a.subboxes) return hipErrorInvalidValue;   // spatial order only
        if (a.tmask && hipMemsetAsync(a.tmask, 0, (size_t)a.T * a.tmw * sizeof(unsigned long long), s) != hipSuccess)
            return hipGetLastError();
        if (variant == 1) {
            if (a.guard) hipLaunchKernelGGL((k_n3b_plan<1, true>), dim3(nplan), dim3(BW * BW), 0, s, a, a.plan);
            else hipLaunchKernelGGL((k_n3b_plan<1, false>), dim3(nplan), dim3(BW * BW), 0, s, a, a.plan);
        } else {
            if (a.guard) hipLaunchKernelGGL((k_n3b_plan<0, true>), dim3(nplan), dim3(BW * BW), 0, s, a, a.plan);
            else hipLaunchKernelGGL((k_n3b_plan<0, false>), dim3(nplan), dim3(BW * BW), 0, s, a, a.plan);
        }
    } else if (a.tailb && !a.plan) {
        return hipErrorInvalidValue;                // the tail sums come from the plan (a rank without blocks: 0)
    }
    return hipGetLastError();
}


hipError_t launch_forces_n3b(const N3BArgs& a, int variant, double* out, hipStream_t s, hipEvent_t ev0, hipEvent_t ev1,
                             hipEvent_t* marks) {
    const int nblk = (a.Phi - a.Plo) * a.R;
    const int nplan = (a.Phi - a.Plo) * a.nd;
    if (hipError_t e = launch_n3b_plan(a, variant, s); e != hipSuccess) return e;
    if (marks && hipEventRecord(marks[0], s) != hipSuccess) return hipGetLastError();
    if (nblk > 0) {
        if (variant == 1 && !a.guard && a.pairs) {   // the paired-wave kernel (option force_n3b_pairs)
            if (n3b_axp(a)) launch_timed(k_pairs_n3b_pw<1, false, false, MDQT_N3B_AX1 != 0>, dim3(nblk), dim3(NWP * 64), s, ev0, ev1, a);
            else launch_timed(k_pairs_n3b_pw<1, false>, dim3(nblk), dim3(NWP * 64), s, ev0, ev1, a);
        } else if (variant == 1) {
            const bool axp = n3b_axp(a);
            if (a.guard) launch_timed(k_pairs_n3b<1, true>, dim3(nblk), dim3(BW * 64), s, ev0, ev1, a);
            else if (axp) launch_timed(k_pairs_n3b<1, false, false, MDQT_N3B_AX1 != 0>, dim3(nblk), dim3(BW * 64), s, ev0, ev1, a);
            else launch_timed(k_pairs_n3b<1, false>, dim3(nblk), dim3(BW * 64), s, ev0, ev1, a);
        } else {
            if (a.guard) launch_timed(k_pairs_n3b<0, true>, dim3(nblk), dim3(BW * 64), s, ev0, ev1, a);
            else launch_timed(k_pairs_n3b<0, false>, dim3(nblk), dim3(BW * 64), s, ev0, ev1, a);
        }
    } else if (ev0) {                                   // (no block of this rank: an empty interval)
        if (hipEventRecord(ev0, s) != hipSuccess || hipEventRecord(ev1, s) != hipSuccess) return hipGetLastError();
    }
    // a rank without blocks (Phi == Plo, sharded with NB < W) has no plan and so no masks to follow:
    // the unmasked reduction reads none of its (unwritten) slots and leaves its dense partial 0
    N3BArgs r = a;
    if (!(a.plan && nplan > 0)) r.tmask = nullptr;
    if (marks && hipEventRecord(marks[1], s) != hipSuccess) return hipGetLastError();
    hipLaunchKernelGGL(k_n3b_reduce, dim3((a.N + 255) / 256, 3), dim3(256), 0, s, r, out);
    if (marks && hipEventRecord(marks[2], s) != hipSuccess) return hipGetLastError();
#if defined(MDQT_EXPT_TMASK_DEBUG)
    if (a.plan && a.tmask) {                        // diagnostic build: the masks' bit counts
        (void)hipStreamSynchronize(s);
        const size_t nj = (size_t)(a.Phi - a.Plo) * a.nd;
        std::vector<uint2> js(nj);
        std::vector<unsigned long long> tm((size_t)a.T * a.tmw);
        (void)hipMemcpy(js.data(), a.plan + nj * (BW * BW), nj * sizeof(uint2), hipMemcpyDeviceToHost);
        (void)hipMemcpy(tm.data(), a.tmask, tm.size() * 8, hipMemcpyDeviceToHost);
        long cj = 0, ct = 0, miss = 0;
        for (size_t k = 0; k < nj; ++k) cj += __builtin_popcount(js[k].x);
        for (auto v : tm) ct += __builtin_popcountll(v);
        for (size_t k = 0; k < nj; ++k) {
            const int P = a.Plo + (int)(k / a.nd), db = (int)(k % a.nd), Q = (P + db) % a.NB;
            for (int b = 0; b < BW; ++b)
                if ((js[k].x >> b) & 1u) {
                    const int J = Q * BW + b;
                    if (!((tm[(size_t)J * a.tmw + (db >> 6)] >> (db & 63)) & 1ull)) ++miss;
                }
        }
        fprintf(stderr, "tmask debug: jstep bits %ld, tmask bits %ld, jstep bits missing in tmask %ld (T %d tmw %d nd %d NB %d)\n",
                cj, ct, miss, a.T, a.tmw, a.nd, a.NB);
    }
#endif
    return hipGetLastError();
}

hipError_t launch_tail_max(const double* tailb, int T, double eps, unsigned long long* st, int* list, hipStream_t s) {
    if (T <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_tail_max, dim3((T + 255) / 256 < 64 ? (T + 255) / 256 : 64), dim3(256), 0, s, tailb, T, eps,
                       st, list);
    return hipGetLastError();
}

hipError_t launch_tail_fix(const N3BArgs& a, const unsigned long long* st, const int* list, double* out,
                           hipStream_t s, bool pot) {
    if (a.T <= 0 || !a.Rs || !a.perm || !a.boxes) return hipErrorInvalidValue;   // spatial order only
    if (pot) hipLaunchKernelGGL(k_tail_fix<true>, dim3(a.T < 512 ? a.T : 512), dim3(256), 0, s, a, st, list, out);
    else hipLaunchKernelGGL(k_tail_fix<false>, dim3(a.T < 512 ? a.T : 512), dim3(256), 0, s, a, st, list, out);
    return hipGetLastError();
}

hipError_t launch_n3b_census(const N3BArgs& a, unsigned long long* out, hipStream_t s, unsigned long long* bw,
                             unsigned long long* bal) {
    if (!a.use_sort || !a.boxes || !a.subboxes) return hipErrorInvalidValue;   // the classes need the boxes
    const int nblk = (a.Phi - a.Plo) * a.nd;
    if (hipMemsetAsync(out, 0, 2 * kCensus * sizeof(unsigned long long), s) != hipSuccess) return hipGetLastError();
    if (bw && a.Phi > a.Plo && hipMemsetAsync(bw, 0, (size_t)(a.Phi - a.Plo) * sizeof(unsigned long long), s) != hipSuccess)
        return hipGetLastError();
    if (bal && hipMemsetAsync(bal, 0, 11 * sizeof(unsigned long long), s) != hipSuccess) return hipGetLastError();
    if (nblk > 0) hipLaunchKernelGGL(k_n3b_census, dim3(nblk), dim3(BW * BW), 0, s, a, out, bw, bal);
    return hipGetLastError();
}

// Epotential()'s pair sums on the blocks.  With a plan (a.plan, the fast variant in spatial order; round
// 6): the force call's skip radius, sub-tile groups and error-bounded forms (pair_u_cut, the f32
// ultra-far form), the tail sums in a.tailb for the caller's enforcement; without: every pair to L/2 in
// the exact form (the staging lanes classify)
hipError_t launch_potential_n3b(const N3BArgs& a, int variant, double* out, hipStream_t s, hipEvent_t ev0,
                                hipEvent_t ev1) {
    if (variant < 0 || variant > 1) return hipErrorInvalidValue;
    const int nblk = (a.Phi - a.Plo) * a.R;
    const int nplan = (a.Phi - a.Plo) * a.nd;
    const bool planned = a.plan && nplan > 0;
    if (planned && (variant != 1 || a.guard)) return hipErrorInvalidValue;   // (the far forms are the fast variant's)
    if (hipError_t e = launch_n3b_plan(a, variant, s); e != hipSuccess) return e;
    N3BArgs r = a;
    if (!planned) { r.plan = nullptr; r.tmask = nullptr; }   // (no plan: every j-slot written, every one read)
    if (nblk > 0) {
        if (variant == 1 && !a.guard && a.pairs) {   // the paired-wave kernel (option force_n3b_pairs)
            if (planned && n3b_axp(a))
                launch_timed(k_pairs_n3b_pw<1, false, true, MDQT_N3B_AX1 != 0>, dim3(nblk), dim3(NWP * 64), s, ev0, ev1, r);
            else launch_timed(k_pairs_n3b_pw<1, false, true>, dim3(nblk), dim3(NWP * 64), s, ev0, ev1, r);
        } else if (variant == 1) {
            if (a.guard) launch_timed(k_pairs_n3b<1, true, true>, dim3(nblk), dim3(BW * 64), s, ev0, ev1, r);
            else if (planned && n3b_axp(a))
                launch_timed(k_pairs_n3b<1, false, true, MDQT_N3B_AX1 != 0>, dim3(nblk), dim3(BW * 64), s, ev0, ev1, r);
            else launch_timed(k_pairs_n3b<1, false, true>, dim3(nblk), dim3(BW * 64), s, ev0, ev1, r);
        } else {
            if (a.guard) launch_timed(k_pairs_n3b<0, true, true>, dim3(nblk), dim3(BW * 64), s, ev0, ev1, r);
            else launch_timed(k_pairs_n3b<0, false, true>, dim3(nblk), dim3(BW * 64), s, ev0, ev1, r);
        }
    } else if (ev0) {
        if (hipEventRecord(ev0, s) != hipSuccess || hipEventRecord(ev1, s) != hipSuccess) return hipGetLastError();
    }
    hipLaunchKernelGGL(k_n3b_reduce, dim3((a.N + 255) / 256, 1), dim3(256), 0, s, r, out);   // component 0
    return hipGetLastError();
}

hipError_t launch_sum_rank_chunks(const double* const* parts, int world, int rank, int S, double* F, hipStream_t s) {
    hipLaunchKernelGGL(k_sum_rank_chunks, dim3((3 * S + 255) / 256), dim3(256), 0, s, parts, world, rank, S, F);
    return hipGetLastError();
}

}  // namespace mdqt
