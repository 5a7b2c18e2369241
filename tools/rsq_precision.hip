// v_rsq_f64 precision probe: max relative error of the raw instruction and after one and two
// Newton steps, against a long-double reference computed on the host; and v_rsq_f32 on the same
// inputs rounded to float (the f32 ultra-far pair form's kRsqF32RelErr, mdqt_internal.hpp).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>

__global__ void kf(const float* x, float* r, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) r[i] = __builtin_amdgcn_rsqf(x[i]);
}

__global__ void k(const double* x, double* r0, double* r1, double* r2, double* r3, int n) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const double v = x[i];
    double r = __builtin_amdgcn_rsq(v);
    r0[i] = r;
    const double hx = 0.5 * v;
    r = r * fma(-hx * r, r, 1.5);
    r1[i] = r;
    r = r * fma(-hx * r, r, 1.5);
    r2[i] = r;
    // one third-order step: r (1 + e/2 + 3e^2/8), e = 1 - x r^2
    const double q = __builtin_amdgcn_rsq(v);
    const double e = fma(-v, q * q, 1.0);
    r3[i] = fma(q * e, fma(e, 0.375, 0.5), q);
}

int main() {
    const int n = 1 << 22;
    double *x = (double*)malloc(n * 8), *h0 = (double*)malloc(n * 8), *h1 = (double*)malloc(n * 8), *h2 = (double*)malloc(n * 8), *h3 = (double*)malloc(n * 8);
    srand48(7);
    for (int i = 0; i < n; ++i) x[i] = exp(log(1e-4) + drand48() * (log(1e6) - log(1e-4)));
    double *dx, *d0, *d1, *d2, *d3;
    hipMalloc(&dx, n * 8); hipMalloc(&d0, n * 8); hipMalloc(&d1, n * 8); hipMalloc(&d2, n * 8); hipMalloc(&d3, n * 8);
    hipMemcpy(dx, x, n * 8, hipMemcpyHostToDevice);
    hipLaunchKernelGGL(k, dim3(n / 256), dim3(256), 0, 0, dx, d0, d1, d2, d3, n);
    hipMemcpy(h0, d0, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(h1, d1, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(h2, d2, n * 8, hipMemcpyDeviceToHost);
    hipMemcpy(h3, d3, n * 8, hipMemcpyDeviceToHost);
    long double e0 = 0, e1 = 0, e2 = 0, e3 = 0;
    for (int i = 0; i < n; ++i) {
        const long double ref = 1.0L / sqrtl((long double)x[i]);
        e0 = fmaxl(e0, fabsl(h0[i] / ref - 1));
        e1 = fmaxl(e1, fabsl(h1[i] / ref - 1));
        e2 = fmaxl(e2, fabsl(h2[i] / ref - 1));
        e3 = fmaxl(e3, fabsl(h3[i] / ref - 1));
    }
    printf("third-order step: %.3Le (2^%.1f)\n", e3, (double)log2l(e3));
    {
        float *xf = (float*)malloc(n * 4), *hf = (float*)malloc(n * 4), *dxf, *drf;
        for (int i = 0; i < n; ++i) xf[i] = (float)x[i];
        hipMalloc(&dxf, n * 4); hipMalloc(&drf, n * 4);
        hipMemcpy(dxf, xf, n * 4, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(kf, dim3(n / 256), dim3(256), 0, 0, dxf, drf, n);
        hipMemcpy(hf, drf, n * 4, hipMemcpyDeviceToHost);
        long double ef = 0;
        for (int i = 0; i < n; ++i) ef = fmaxl(ef, fabsl(hf[i] * sqrtl((long double)xf[i]) - 1));
        printf("rsq_f32: %.3Le (2^%.1f)\n", ef, (double)log2l(ef));
    }
    printf("max rel err: raw %.3Le (2^%.1f)  1 NR %.3Le (2^%.1f)  2 NR %.3Le (2^%.1f)\n", e0, (double)log2l(e0), e1,
           (double)log2l(e1), e2, (double)log2l(e2));
    return 0;
}
