// Diagnostic (not product code): how fast the dispatcher starts the workgroups of a grid shaped
// like the C2 Newton-3 tile kernel (1,596 workgroups x 256 threads, 22.5 KB LDS, 65 VGPRs), and
// whether busy CUs slow it down.  Each workgroup stamps s_memrealtime (100 MHz) at entry and exit;
// its waves then run `iters` iterations of 4 independent FP64 FMA chains (iters = 0: empty body).
//   hipcc --offload-arch=gfx950 -O3 -o tools/dispatch_probe tools/dispatch_probe.hip
//   tools/dispatch_probe [grid] [iters...]
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

__global__ __launch_bounds__(256) void k_probe(unsigned long long* st, int iters, double* sink) {
    extern __shared__ double lds[];
    const unsigned long long t0 = __builtin_amdgcn_s_memrealtime();
    double a = threadIdx.x * 1e-3, b = a + 1., c = a + 2., d = a + 3.;
    for (int i = 0; i < iters; ++i) {
        a = fma(a, 0.999999, 1e-7);
        b = fma(b, 0.999999, 1e-7);
        c = fma(c, 0.999999, 1e-7);
        d = fma(d, 0.999999, 1e-7);
    }
    lds[threadIdx.x] = a + b + c + d;
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memrealtime();
        st[4 * blockIdx.x] = t0;
        st[4 * blockIdx.x + 1] = t1;
        st[4 * blockIdx.x + 2] = __builtin_amdgcn_s_getreg((31 << 11) | 4);   // HW_ID
        st[4 * blockIdx.x + 3] = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // XCC_ID
        if (lds[1] == 12345.) sink[0] = lds[2];
    }
}

static double pct(std::vector<double> v, double p) {
    std::sort(v.begin(), v.end());
    return v[(size_t)(p / 100. * (v.size() - 1))];
}

int main(int argc, char** argv) {
    const int grid = argc > 1 ? atoi(argv[1]) : 1596;
    std::vector<int> its;
    for (int k = 2; k < argc; ++k) its.push_back(atoi(argv[k]));
    if (its.empty()) its = {0, 200, 2000};
    unsigned long long* d;
    double* sink;
    CHK(hipMalloc(&d, sizeof(unsigned long long) * 4 * grid));
    CHK(hipMalloc(&sink, 8));
    std::vector<unsigned long long> h(4 * grid);
    for (int it : its) {
        for (int rep = 0; rep < 3; ++rep) {
            hipLaunchKernelGGL(k_probe, dim3(grid), dim3(256), 22528, 0, d, it, sink);
            CHK(hipDeviceSynchronize());
        }
        CHK(hipMemcpy(h.data(), d, h.size() * 8, hipMemcpyDeviceToHost));
        unsigned long long t0 = ~0ull;
        for (int b = 0; b < grid; ++b) t0 = std::min(t0, h[4 * b]);
        std::vector<double> s(grid), e(grid);
        double corr = 0;
        for (int b = 0; b < grid; ++b) {
            s[b] = (h[4 * b] - t0) * 1e-2;
            e[b] = (h[4 * b + 1] - t0) * 1e-2;
            corr += s[b] * b;
        }
        printf("iters %5d grid %d: start us p0/10/50/90/100 %.2f %.2f %.2f %.2f %.2f | end p50/100 %.2f %.2f | "
               "start of block grid/2: %.2f, of the last block: %.2f\n",
               it, grid, pct(s, 0), pct(s, 10), pct(s, 50), pct(s, 90), pct(s, 100), pct(e, 50), pct(e, 100),
               s[grid / 2], s[grid - 1]);
    }
    return 0;
}
