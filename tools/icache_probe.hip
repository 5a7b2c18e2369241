// Diagnostic (not product code): what a cold instruction cache costs a wave on gfx950.  Each wave
// runs a straight-line block of KB kilobytes of independent v_fma_f64 (8 bytes each, 4 chains) twice
// (a non-unrolled loop: the same code addresses), stamping s_memtime around each pass; the first pass
// pays the instruction fetches, the second runs from the instruction cache.  The kernel is launched
// twice back to back, so the first pass of the second launch shows whether a launch starts cold.
//   hipcc --offload-arch=gfx950 -O3 -o tools/icache_probe tools/icache_probe.hip && tools/icache_probe
#include <hip/hip_runtime.h>

#include <algorithm>
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

#define F4 "v_fma_f64 %0, %4, %5, %0\n v_fma_f64 %1, %4, %5, %1\n v_fma_f64 %2, %4, %5, %2\n v_fma_f64 %3, %4, %5, %3\n"
#define F16 F4 F4 F4 F4
#define F64 F16 F16 F16 F16
#define F256 F64 F64 F64 F64   // 2 KB of code

__device__ __forceinline__ void blk2k(double& a, double& b, double& c, double& d, double x, double y) {
    asm volatile(F256 : "+v"(a), "+v"(b), "+v"(c), "+v"(d) : "v"(x), "v"(y));
}

template <int KB2>   // number of 2 KB blocks
__global__ __launch_bounds__(256) void k_icache(unsigned long long* st, double* sink) {
    double a = threadIdx.x * 1e-3, b = a + 1., c = a + 2., d = a + 3.;
    const double x = 0.999999, y = 1e-7;
    unsigned long long t[3];
#pragma nounroll
    for (int pass = 0; pass < 2; ++pass) {
        t[pass] = __builtin_amdgcn_s_memtime();
#pragma unroll
        for (int r = 0; r < KB2; ++r) blk2k(a, b, c, d, x, y);
    }
    t[2] = __builtin_amdgcn_s_memtime();
    const int wv = blockIdx.x * 4 + (threadIdx.x >> 6), l = threadIdx.x & 63;
    if (l < 2) st[2 * wv + l] = l == 0 ? t[1] - t[0] : t[2] - t[1];   // vector stores
    if (a + b + c + d == 12345.678) sink[0] = a;
}

template <int KB2>
static void run(int grid) {
    const int nw = grid * 4;
    unsigned long long* st;
    double* sink;
    CHK(hipMalloc(&st, sizeof(unsigned long long) * 2 * nw));
    CHK(hipMalloc(&sink, 8));
    std::vector<unsigned long long> h(2 * nw);
    for (int launch = 0; launch < 3; ++launch) {
        hipLaunchKernelGGL(k_icache<KB2>, dim3(grid), dim3(256), 0, 0, st, sink);
        CHK(hipDeviceSynchronize());
        CHK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
        std::vector<unsigned long long> p0(nw), p1(nw);
        for (int w = 0; w < nw; ++w) { p0[w] = h[2 * w]; p1[w] = h[2 * w + 1]; }
        std::sort(p0.begin(), p0.end());
        std::sort(p1.begin(), p1.end());
        printf("code %3d KB  grid %4d  launch %d: pass1 cycles med %7llu max %7llu | pass2 med %7llu max %7llu"
               " | cold extra med %6lld (%.1f per 64 B line)\n",
               2 * KB2, grid, launch, p0[nw / 2], p0[nw - 1], p1[nw / 2], p1[nw - 1],
               (long long)p0[nw / 2] - (long long)p1[nw / 2],
               ((double)p0[nw / 2] - (double)p1[nw / 2]) / (KB2 * 2048 / 64.));
    }
    CHK(hipFree(st));
    CHK(hipFree(sink));
}

int main() {
    for (int grid : {1, 256}) {
        run<1>(grid);
        run<4>(grid);
        run<8>(grid);
        run<16>(grid);
    }
    return 0;
}
