// v_exp_f32 precision probe (the ultra-far pair form's bound assumes it, mdqt_internal.hpp
// kExp2fRelErr): max relative error of __builtin_amdgcn_exp2f(x) over x in [-70, 0] (2^-70 ~ 8e-22,
// inside f32's normal range) against a long-double reference of 2^x at the same float x.
//   hipcc --offload-arch=gfx950 -O3 tools/exp2f_precision.hip -o tools/exp2f_precision
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void k(const float* x, float* y, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) y[i] = __builtin_amdgcn_exp2f(x[i]);
}

int main() {
    const int n = 1 << 24;
    float* x = (float*)malloc(n * 4);
    float* y = (float*)malloc(n * 4);
    srand48(11);
    for (int i = 0; i < n; ++i) x[i] = (float)(-70.0 * drand48());
    x[0] = 0.f; x[1] = -70.f; x[2] = -0.5f; x[3] = -1e-7f;
    float *dx, *dy;
    if (hipMalloc(&dx, n * 4) != hipSuccess || hipMalloc(&dy, n * 4) != hipSuccess) return 1;
    hipMemcpy(dx, x, n * 4, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dx, dy, n);
    hipMemcpy(y, dy, n * 4, hipMemcpyDeviceToHost);
    long double e = 0;
    for (int i = 0; i < n; ++i) {
        const long double ref = exp2l((long double)x[i]);
        const long double r = fabsl((long double)y[i] / ref - 1);
        if (r > e) e = r;
    }
    printf("max rel err exp2f: %.3Le (2^%.2f)\n", e, (double)log2l(e));
    return 0;
}
