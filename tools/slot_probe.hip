// Diagnostic (not product code): what the QT launch's prologue pays for the 56 Newton-3 force
// slots at C2, by slot layout.  A writer kernel stores the slots the way the tile kernel does (one
// 4-wave workgroup per tile pair, write-through stores of 64 rows x 3 components into two slots),
// then a reader kernel shaped like the lane kernel's prologue (16 lanes per ion, lane k sums
// slots k, k+16, k+32, k+48 of the 3 components, 16-lane tree, F stored) is timed with events.
//   layout 0: [slot][3][S]           (the product's)
//   layout 1: [slot/16][3][S][16]    (an ion's 16 lanes read one 128-byte line per round)
//   layout 2: F only                 (3 loads per ion: the floor without slots)
//   hipcc --offload-arch=gfx950 -O3 -o tools/slot_probe tools/slot_probe.hip && tools/slot_probe
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

#define CHK(x)                                                                              \
    do {                                                                                    \
        hipError_t e_ = (x);                                                                \
        if (e_ != hipSuccess) {                                                             \
            fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_));       \
            exit(1);                                                                        \
        }                                                                                   \
    } while (0)

constexpr int N = 3573, S = 3584, T = 56;

__device__ __forceinline__ size_t addr(int layout, int s, int c, int i) {
    if (layout == 1) return ((((size_t)(s >> 4) * 3 + c) * S + i) << 4) + (s & 15);
    return ((size_t)s * 3 + c) * S + i;
}

__device__ __forceinline__ void wt_store(double* p, double v) {
    __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}

template <int layout>
__global__ __launch_bounds__(256) void k_write(double* P, double* F0, const int2* pairs, double salt) {
    const int2 IJ = pairs[blockIdx.x];
    const int q = threadIdx.x >> 6, l = threadIdx.x & 63;
    if (q == 0) {
        const int i = IJ.x * 64 + l;
        if (i < S)
            for (int c = 0; c < 3; ++c) wt_store(&P[addr(layout == 1 ? 1 : 0, IJ.y, c, i)], salt + i * 1e-3 + c + IJ.y);
    } else if (q == 1 && IJ.x != IJ.y) {
        const int j = IJ.y * 64 + l;
        if (j < S)
            for (int c = 0; c < 3; ++c) wt_store(&P[addr(layout == 1 ? 1 : 0, IJ.x, c, j)], salt + j * 1e-3 + c + IJ.x);
    } else if (q == 2 && IJ.x == IJ.y) {                // F itself (layout 2's input), also write-through
        const int i = IJ.x * 64 + l;
        if (i < S)
            for (int c = 0; c < 3; ++c) wt_store(&F0[(size_t)c * S + i], salt + i * 1e-3 + c);
    }
}

template <int layout>
__global__ __launch_bounds__(256) void k_read(const double* __restrict__ P, const double* __restrict__ F0,
                                              double* F) {
    const int k = threadIdx.x & 15;
    const int i = min(blockIdx.x * 16 + (threadIdx.x >> 4), N - 1);
    double q[3] = {0., 0., 0.};
    if (layout == 2) {
        if (k < 3) q[k] = F0[(size_t)k * S + i];
    } else {
        double t[4][3];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
            const int s = min(k + 16 * u, T - 1);
#pragma unroll
            for (int c = 0; c < 3; ++c) t[u][c] = P[addr(layout, s, c, i)];
        }
#pragma unroll
        for (int u = 0; u < 4; ++u)
#pragma unroll
            for (int c = 0; c < 3; ++c) q[c] += (k + 16 * u < T) ? t[u][c] : 0.;
    }
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        double v = q[c];
        for (int o = 1; o < 16; o <<= 1) v += __shfl_xor(v, o, 16);
        q[c] = v;
    }
    if (k < 3) F[(size_t)k * S + i] = q[k];
}

__global__ __launch_bounds__(256) void k_empty(double* F) {
    if (threadIdx.x == 1000) F[0] = 1.;
}
template <int X>
__global__ __launch_bounds__(256) void k_read_again(const double* __restrict__ F0, double* F) {   // F0 L2-warm
    const int k = threadIdx.x & 15;
    const int i = min(blockIdx.x * 16 + (threadIdx.x >> 4), N - 1);
    if (k < 3) F[(size_t)k * S + i] = F0[(size_t)k * S + i] * 2.;
}

int main() {
    std::vector<int2> pairs;
    for (int I = 0; I < T; ++I)
        for (int J = I + 1; J < T; ++J) pairs.push_back({I, J});
    for (int I = 0; I < T; ++I) pairs.push_back({I, I});
    int2* dp;
    double *P, *F, *F0;
    const size_t n = (size_t)T * 3 * S + 64 * 3 * S;
    CHK(hipMalloc(&dp, pairs.size() * sizeof(int2)));
    CHK(hipMemcpy(dp, pairs.data(), pairs.size() * sizeof(int2), hipMemcpyHostToDevice));
    CHK(hipMalloc(&P, n * 8));
    CHK(hipMalloc(&F, 3 * S * 8));
    CHK(hipMalloc(&F0, 3 * S * 8));
    CHK(hipMemset(P, 0, n * 8));
    CHK(hipMemset(F0, 0, 3 * S * 8));
    hipEvent_t e0, e1, e2;
    CHK(hipEventCreate(&e2));
    CHK(hipEventCreate(&e0));
    CHK(hipEventCreate(&e1));
    const int reps = 400;
    for (int round = 0; round < 3; ++round) {
        for (int layout = 0; layout < 3; ++layout) {
            double tot = 0., wtot = 0.;
            float best = 1e9;
            for (int r = 0; r < reps; ++r) {
                CHK(hipEventRecord(e2, 0));
                if (layout == 1) hipLaunchKernelGGL(k_write<1>, dim3(pairs.size()), dim3(256), 0, 0, P, F0, dp, (double)r);
                else if (layout == 0) hipLaunchKernelGGL(k_write<0>, dim3(pairs.size()), dim3(256), 0, 0, P, F0, dp, (double)r);
                else hipLaunchKernelGGL(k_write<2>, dim3(pairs.size()), dim3(256), 0, 0, P, F0, dp, (double)r);
                CHK(hipEventRecord(e0, 0));
                if (layout == 0) hipLaunchKernelGGL(k_read<0>, dim3((N + 15) / 16), dim3(256), 0, 0, P, F0, F);
                else if (layout == 1) hipLaunchKernelGGL(k_read<1>, dim3((N + 15) / 16), dim3(256), 0, 0, P, F0, F);
                else hipLaunchKernelGGL(k_read<2>, dim3((N + 15) / 16), dim3(256), 0, 0, P, F0, F);
                CHK(hipEventRecord(e1, 0));
                CHK(hipEventSynchronize(e1));
                float ms;
                CHK(hipEventElapsedTime(&ms, e0, e1));
                float wms;
                CHK(hipEventElapsedTime(&wms, e2, e0));
                if (r >= 20) { tot += ms; wtot += wms; }
                if (ms < best) best = ms;
            }
            printf("round %d layout %d: reader mean %.2f us  min %.2f us   writer mean %.2f us\n", round, layout,
                   tot / (reps - 20) * 1e3, best * 1e3, wtot / (reps - 20) * 1e3);
        }
    }
    for (int r = 0; r < 400; ++r) {   // floors: an empty launch; F read twice in a row (no writer between)
        hipLaunchKernelGGL(k_empty, dim3((N + 15) / 16), dim3(256), 0, 0, F);
        hipLaunchKernelGGL(k_read_again<0>, dim3((N + 15) / 16), dim3(256), 0, 0, F0, F);
        hipLaunchKernelGGL(k_read_again<1>, dim3((N + 15) / 16), dim3(256), 0, 0, F0, F);
    }
    CHK(hipDeviceSynchronize());
    return 0;
}
