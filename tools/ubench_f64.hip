// Microbenchmark (diagnostic tool, not product): FP64 VALU issue cost and dependent latency on
// gfx950, per wave, from s_memtime around an unrolled loop.  Shapes the QT-kernel layout
// (DESIGN.md §3): how many independent chains / waves per SIMD a dependent FP64 stream needs.
//   hipcc --offload-arch=gfx950 -O3 -o tools/ubench_f64 tools/ubench_f64.hip
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <vector>
#include <algorithm>
#include <stdlib.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

template <int CTRL>
__device__ __forceinline__ double dppd(double v) {
    const int lo = __builtin_amdgcn_update_dpp(0, __double2loint(v), CTRL, 0xF, 0xF, true);
    const int hi = __builtin_amdgcn_update_dpp(0, __double2hiint(v), CTRL, 0xF, 0xF, true);
    return __hiloint2double(hi, lo);
}

// OP 0: fma f64; 1: add f64; 2: fma f32; 3: x = x + dpp_ror8(x) (2 movs + add); 4: rsq f64 + fma;
// 5: mul f64; 6: packed fma f32 (v_pk_fma_f32); 7: packed mul f32 (v_pk_mul_f32); 8: exp f32 + fma f32;
// 9: rsq f32 + fma f32; (round 6, the block kernel's far forms) 10: cvt f64->f32->f64 + fma f64; 11: rndne f64 +
// fma f64; 12: cvt_i32_f64 + ldexp f64; 13: exp f32 between conversions + fma f64 (the ultra-far form's 2^t);
// 14: rsq f64 alone (x = rsq(x)); 15: ldexp f64 + fma f64
typedef float f32x2 __attribute__((ext_vector_type(2)));
template <int OP, int CH>
__global__ __launch_bounds__(256) void k(double* out, long long* cyc, int iters, double a, double b) {
    const int gid = blockIdx.x * 256 + threadIdx.x;
    double x[CH];
    float xf[CH];
    f32x2 xp[CH];
#pragma unroll
    for (int c = 0; c < CH; ++c) { x[c] = threadIdx.x * 1e-3 + c; xf[c] = (float)x[c]; xp[c] = f32x2{xf[c], xf[c] + 1.f}; }
    const float af = (float)a, bf = (float)b;
    __builtin_amdgcn_s_waitcnt(0);
    const long long t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < iters; ++it) {
#pragma unroll
        for (int r = 0; r < 16; ++r) {
#pragma unroll
            for (int c = 0; c < CH; ++c) {
                if (OP == 0) x[c] = fma(x[c], a, b);
                else if (OP == 1) x[c] = x[c] + a;
                else if (OP == 2) xf[c] = fmaf(xf[c], af, bf);
                else if (OP == 3) x[c] = x[c] * a + dppd<0x128>(x[c]);
                else if (OP == 4) x[c] = fma(__builtin_amdgcn_rsq(x[c]), a, b);
                else if (OP == 6) xp[c] = __builtin_elementwise_fma(xp[c], f32x2{af, af}, f32x2{bf, bf});
                else if (OP == 7) xp[c] = xp[c] * f32x2{af, bf};
                else if (OP == 8) xf[c] = fmaf(__builtin_amdgcn_exp2f(xf[c]), af, -bf);
                else if (OP == 9) xf[c] = fmaf(__builtin_amdgcn_rsqf(xf[c]), af, bf);
                else if (OP == 10) x[c] = fma((double)(float)x[c], a, b);
                else if (OP == 11) x[c] = fma(__builtin_rint(x[c]), a, b);
                else if (OP == 12) x[c] = ldexp(x[c], ((int)x[c] & 1) - 1);
                else if (OP == 13) x[c] = fma((double)__builtin_amdgcn_exp2f((float)x[c]), a, -b);
                else if (OP == 14) x[c] = __builtin_amdgcn_rsq(x[c]);
                else if (OP == 15) x[c] = fma(ldexp(x[c], -1), a, b);
                else x[c] = x[c] * a;
            }
        }
    }
    const long long t1 = __builtin_amdgcn_s_memtime();
    double s = 0;
#pragma unroll
    for (int c = 0; c < CH; ++c) s += x[c] + xf[c] + xp[c].x + xp[c].y;
    out[gid] = s;
    cyc[gid] = t1 - t0;
}

template <int OP, int CH>
static int run(const char* name, int wps, double* dout, long long* dcyc, int iters) {
    const int blocks = 256 * wps;   // 256-thread blocks: one wave per SIMD per block
    hipLaunchKernelGGL((k<OP, CH>), dim3(blocks), dim3(256), 0, 0, dout, dcyc, iters, 0.999999, 1e-7);
    CHK(hipDeviceSynchronize());
    hipEvent_t e0, e1;
    hipEventCreate(&e0); hipEventCreate(&e1);
    hipEventRecord(e0);
    hipLaunchKernelGGL((k<OP, CH>), dim3(blocks), dim3(256), 0, 0, dout, dcyc, iters, 0.999999, 1e-7);
    hipEventRecord(e1);
    CHK(hipDeviceSynchronize());
    float ms = 0; hipEventElapsedTime(&ms, e0, e1);
    std::vector<long long> c((size_t)blocks * 256);
    CHK(hipMemcpy(c.data(), dcyc, c.size() * sizeof(long long), hipMemcpyDeviceToHost));
    std::vector<long long> w;
    for (size_t i = 0; i < c.size(); i += 64) w.push_back(c[i]);
    std::sort(w.begin(), w.end());
    const double ninst = (double)iters * 16 * CH;   // per wave
    const double med = (double)w[w.size() / 2];
    const double total_inst = ninst * blocks * 4;   // waves
    printf("%-10s CH=%d wps=%d  cyc/inst/wave(median)=%.2f  SIMD-cycles/inst=%.2f  wall=%.3f ms  clk_est=%.2f GHz\n",
           name, CH, wps, med / ninst, med / ninst / wps, ms, total_inst / 1024.0 * (med / ninst / wps) / (ms * 1e-3) / 1e9);
    return 0;
}

int main() {
    double* dout; long long* dcyc;
    const int maxb = 256 * 8;
    CHK(hipMalloc(&dout, (size_t)maxb * 256 * sizeof(double)));
    CHK(hipMalloc(&dcyc, (size_t)maxb * 256 * sizeof(long long)));
    const int it = 2000;
    if (getenv("UBENCH_FORMS")) {                  // round 6: the far forms' instructions, throughput
        run<0, 4>("fma_f64", 4, dout, dcyc, it);
        run<5, 4>("mul_f64", 4, dout, dcyc, it);
        run<1, 4>("add_f64", 4, dout, dcyc, it);
        run<2, 4>("fma_f32", 4, dout, dcyc, it);
        run<6, 4>("pkfma_f32", 4, dout, dcyc, it);
        run<10, 4>("cvt2+fma", 4, dout, dcyc, it / 4);
        run<11, 4>("rndne+fma", 4, dout, dcyc, it / 4);
        run<12, 4>("cvti+ldexp", 4, dout, dcyc, it / 4);
        run<15, 4>("ldexp+fma", 4, dout, dcyc, it / 4);
        run<13, 4>("cvt-exp-cvt+fma", 4, dout, dcyc, it / 4);
        run<14, 4>("rsq_f64", 4, dout, dcyc, it / 4);
        run<4, 4>("rsq+fma", 4, dout, dcyc, it / 4);
        run<8, 4>("exp+fma32", 4, dout, dcyc, it / 4);
        run<9, 4>("rsq+fma32", 4, dout, dcyc, it / 4);
        run<3, 4>("dpp+fma", 4, dout, dcyc, it);
        return 0;
    }
    for (int wps : {1, 2, 4}) {
        run<0, 1>("fma_f64", wps, dout, dcyc, it);
        run<0, 2>("fma_f64", wps, dout, dcyc, it);
        run<0, 4>("fma_f64", wps, dout, dcyc, it);
        run<0, 8>("fma_f64", wps, dout, dcyc, it);
        run<1, 1>("add_f64", wps, dout, dcyc, it);
        run<1, 4>("add_f64", wps, dout, dcyc, it);
        run<5, 1>("mul_f64", wps, dout, dcyc, it);
        run<5, 4>("mul_f64", wps, dout, dcyc, it);
        run<2, 1>("fma_f32", wps, dout, dcyc, it);
        run<2, 4>("fma_f32", wps, dout, dcyc, it);
        run<3, 1>("dpp+fma", wps, dout, dcyc, it);
        run<3, 4>("dpp+fma", wps, dout, dcyc, it);
        run<4, 1>("rsq+fma", wps, dout, dcyc, it / 4);
        run<4, 4>("rsq+fma", wps, dout, dcyc, it / 4);
        run<2, 8>("fma_f32", wps, dout, dcyc, it);
        run<6, 1>("pkfma_f32", wps, dout, dcyc, it);
        run<6, 4>("pkfma_f32", wps, dout, dcyc, it);
        run<6, 8>("pkfma_f32", wps, dout, dcyc, it);
        run<7, 4>("pkmul_f32", wps, dout, dcyc, it);
        run<7, 8>("pkmul_f32", wps, dout, dcyc, it);
        run<8, 4>("exp+fma32", wps, dout, dcyc, it / 4);
        run<9, 4>("rsq+fma32", wps, dout, dcyc, it / 4);
    }
    return 0;
}
