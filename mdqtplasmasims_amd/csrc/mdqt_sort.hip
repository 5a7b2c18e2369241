// Spatial ordering for the Newton-3 block-pair force kernel (N > 65,536; SURVEY §8 a1 at C3-C5).
//
// forces() keeps a pair only if its minimum-image separation is below L/2 (SpeedUp:222): about
// 1 - pi/6 = 48 % of all pairs contribute exactly 0.  Evaluated in the ions' storage order, every
// 64-ion tile is spread over the whole box and no tile pair can be skipped.  Ordered along a
// Hilbert curve, a tile occupies a compact region (about 7.5 x 7.5 x 7.5 at the reference's
// density), so a tile pair whose bounding boxes are at least L/2 apart in the minimum image
// contributes nothing and is skipped whole by k_pairs_n3b.
//
//   k_curve_keys    30-bit Hilbert key of every ion (10 bits per axis of x / L)
//   sort_pairs       hipCUB radix sort (key, ion): stable, so every rank of a sharded run that
//                    sorts the same gathered positions gets the same order
//   k_gather_sorted  positions in sorted order, [3][Npad]
//   k_tile_boxes     per 64-ion tile: a reference ion, the minimum-image offsets of the others
//                    from it, their min / max per axis -> center and half extents; the same per
//                    16-ion sub-tile
// Skipped pairs would have added exact zeros, so the forces are bit-identical with and without
// the skipping for a given order (tests/test_gpu_large.py checks it).
#include "mdqt_internal.hpp"

#include <hipcub/hipcub.hpp>

namespace mdqt {

__device__ __forceinline__ uint32_t part1by2(uint32_t x) {   // bits of x spread to every third bit
    x &= 0x3FF;
    x = (x | (x << 16)) & 0x030000FF;
    x = (x | (x << 8)) & 0x0300F00F;
    x = (x | (x << 4)) & 0x030C30C3;
    x = (x | (x << 2)) & 0x09249249;
    return x;
}

__device__ __forceinline__ const double* ion_pos(const double* Rall, int g, int S) {
    const int w = g / S;
    return Rall + (size_t)w * 3 * S + (g - w * S);
}

__global__ __launch_bounds__(256) void k_curve_keys(const double* __restrict__ Rall, int N, int S, double L,
                                                     uint32_t* __restrict__ keys, int* __restrict__ ion) {
    const int g = blockIdx.x * 256 + threadIdx.x;
    if (g >= N) return;
    const double* p = ion_pos(Rall, g, S);
    const double sc = 1024.0 / L;
    uint32_t q[3];
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        double x = p[(size_t)c * S] * sc;
        x = x - 1024.0 * floor(x * (1.0 / 1024.0));          // wrap (positions may sit just outside [0, L))
        int v = (int)x;
        q[c] = (uint32_t)(v < 0 ? 0 : v > 1023 ? 1023 : v);
    }
    // Hilbert index (Skilling's transpose form, 10 bits per axis): consecutive cells are always
    // face neighbours, so a run of 64 ions spans ~1-2 cells — tiles ~3.7 in half extent per axis
    // at the reference's density where the Morton order (jumps at every octant boundary) gives
    // 6.2 x 4.6 x 3.7, and ~1.5x more tile pairs are skipped (16.7 % vs 11.5 % at C5)
    uint32_t X0 = q[0], X1 = q[1], X2 = q[2];
    for (uint32_t Q = 1u << 9; Q > 1; Q >>= 1) {       // inverse undo
        const uint32_t P = Q - 1;
        if (X0 & Q) X0 ^= P;                            // i = 0: X[0] vs itself
        if (X1 & Q) X0 ^= P; else { const uint32_t t = (X0 ^ X1) & P; X0 ^= t; X1 ^= t; }
        if (X2 & Q) X0 ^= P; else { const uint32_t t = (X0 ^ X2) & P; X0 ^= t; X2 ^= t; }
    }
    X1 ^= X0; X2 ^= X1;                                 // Gray encode
    uint32_t t = 0;
    for (uint32_t Q = 1u << 9; Q > 1; Q >>= 1)
        if (X2 & Q) t ^= Q - 1;
    X0 ^= t; X1 ^= t; X2 ^= t;
    keys[g] = part1by2(X2) | (part1by2(X1) << 1) | (part1by2(X0) << 2);
    ion[g] = g;
}

__global__ __launch_bounds__(256) void k_gather_sorted(const double* __restrict__ Rall, int N, int S, int Npad,
                                                       const int* __restrict__ perm, double* __restrict__ Rs) {
    const int t = blockIdx.x * 256 + threadIdx.x;
    if (t >= Npad) return;
    if (t < N) {
        const double* p = ion_pos(Rall, perm[t], S);
        Rs[t] = p[0];
        Rs[(size_t)Npad + t] = p[S];
        Rs[2 * (size_t)Npad + t] = p[2 * (size_t)S];
    } else {                                               // padding of the ragged last tile: the block
        const double pad = (double)((t & 63) + 1) * 0x1p-10;   // kernel's pad ions (distinct points, weight 0),
        Rs[t] = pad; Rs[(size_t)Npad + t] = pad; Rs[2 * (size_t)Npad + t] = pad;   // staged as they are
    }
}

// one wave per tile; boxes[c][T] = center, boxes[3 + c][T] = half extent (+ a rounding margin),
// boxes[6 + c][T] / boxes[9 + c][T] = min / max of the raw coordinates (exact; for the tile pair's
// uniform minimum image in k_pairs_n3b); sub (if not null) [6][4T]: center and half extent of the
// tile's four 16-ion sub-tiles (k_pairs_n3b's sub-tile groups and tail sums)
__global__ __launch_bounds__(256) void k_tile_boxes(const double* __restrict__ Rs, int N, int Npad, int T, double L,
                                                    double* __restrict__ boxes, double* __restrict__ sub) {
    const int tile = blockIdx.x * 4 + (threadIdx.x >> 6);
    const int l = threadIdx.x & 63;
    if (tile >= T) return;                                 // wave-uniform
    const int j = tile * 64 + l;
    const bool v = j < N;
    const double invL = 1.0 / L;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const double* X = Rs + (size_t)c * Npad;
        const double ref = X[tile * 64];
        double d = v ? X[j] - ref : 0.;
        d = fma(-__builtin_rint(d * invL), L, d);          // minimum-image offset from the reference ion
        double lo = d, hi = d;
        double rl = v ? X[j] : ref, rh = rl;
#pragma unroll
        for (int m = 32; m >= 1; m >>= 1) {
            lo = fmin(lo, __shfl_xor(lo, m));
            hi = fmax(hi, __shfl_xor(hi, m));
            rl = fmin(rl, __shfl_xor(rl, m));
            rh = fmax(rh, __shfl_xor(rh, m));
        }
        if (l == c) {
            boxes[(size_t)c * T + tile] = ref + 0.5 * (lo + hi);
            boxes[(size_t)(3 + c) * T + tile] = 0.5 * (hi - lo) * (1. + 1e-12) + 1e-12 * L;
            boxes[(size_t)(6 + c) * T + tile] = rl;
            boxes[(size_t)(9 + c) * T + tile] = rh;
        }
        if (sub) {                                         // the four 16-ion sub-tiles' boxes, the same
            const double sref = X[tile * 64 + (l & 48)];   // way from each sub-tile's first ion
            double e = v ? X[j] - sref : 0.;
            e = fma(-__builtin_rint(e * invL), L, e);
            double slo = e, shi = e;
#pragma unroll
            for (int m = 8; m >= 1; m >>= 1) {
                slo = fmin(slo, __shfl_xor(slo, m));
                shi = fmax(shi, __shfl_xor(shi, m));
            }
            if ((l & 15) == 0) {
                const int st = 4 * tile + (l >> 4);
                sub[(size_t)c * 4 * T + st] = sref + 0.5 * (slo + shi);
                sub[(size_t)(3 + c) * 4 * T + st] = 0.5 * (shi - slo) * (1. + 1e-12) + 1e-12 * L;
            }
        }
    }
}

hipError_t launch_spatial_order(const SortArgs& a, hipStream_t s) {
    if (a.N <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_curve_keys, dim3((a.N + 255) / 256), dim3(256), 0, s, a.Rall, a.N, a.S, a.L, a.keys,
                       a.ion);
    size_t bytes = a.tmp_bytes;
    hipError_t e = hipcub::DeviceRadixSort::SortPairs(a.tmp, bytes, a.keys, a.keys2, a.ion, a.perm, a.N, 0, 30, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_gather_sorted, dim3((a.Npad + 255) / 256), dim3(256), 0, s, a.Rall, a.N, a.S, a.Npad,
                       a.perm, a.Rs);
    const int T = a.Npad / 64;
    hipLaunchKernelGGL(k_tile_boxes, dim3((T + 3) / 4), dim3(256), 0, s, a.Rs, a.N, a.Npad, T, a.L, a.boxes,
                       a.subboxes);
    return hipGetLastError();
}

size_t spatial_order_tmp_bytes(int N) {
    size_t bytes = 0;
    if (hipcub::DeviceRadixSort::SortPairs(nullptr, bytes, (const uint32_t*)nullptr, (uint32_t*)nullptr,
                                           (const int*)nullptr, (int*)nullptr, N, 0, 30) != hipSuccess)
        return 0;
    return bytes;
}

}  // namespace mdqt
