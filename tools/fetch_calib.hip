// FETCH_SIZE / WRITE_SIZE calibration for the access patterns of the QT launch (MI355X_MICROARCH.md
// §HBM: FETCH_SIZE reads exactly half the bytes of a 16-B-per-lane streaming read on gfx950; "other
// access widths are uncalibrated: calibrate on a known byte count in your own access pattern").
//
//   hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/fetch_calib
//   rocprofv3 --pmc FETCH_SIZE -d out -o run -- tools/fetch_calib      (and a WRITE_SIZE pass)
//
// Kernels (each run 5 times, a 512 MiB scrub write between runs so the bytes come from beyond L2):
//   k_stream16   16 B per lane, coalesced                  known bytes: 64 MiB  (the guide's case)
//   k_stream8    8 B per lane, coalesced                   known bytes: 64 MiB
//   k_slots      the QT prologue's force-slot pattern: a wave = 4 consecutive ions x 16 lanes, lane k
//                reads slots k, k+16, k+32, k+48 (< nslots) of 3 components ([nslots][3][S] doubles,
//                S = 3584, 3573 ions, 56 slots: C2) — known bytes: every 128-B line of the slot
//                planes the 3573 ions cover, once (each line is read by one workgroup of 16 ions)
//   k_state      R, V, tPart, psi reads of the same launch (8 B per lane over 16-lane rows)
//   k_store8     8 B per lane coalesced stores (the state write-back)      known bytes: 64 MiB
// prints the known byte counts; divide the profiler's per-kernel FETCH_SIZE / WRITE_SIZE (kB) by them.
#include <hip/hip_runtime.h>
#include <stdio.h>

#define CHK(x) do { hipError_t e = (x); if (e != hipSuccess) { printf("%s: %s\n", #x, hipGetErrorString(e)); return 1; } } while (0)

__global__ void k_stream16(const double2* __restrict__ p, size_t n, double* out) {
    double acc = 0.;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) { double2 v = p[i]; acc += v.x + v.y; }
    if (acc == 12345.678) out[0] = acc;
}
__global__ void k_stream8(const double* __restrict__ p, size_t n, double* out) {
    double acc = 0.;
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) acc += p[i];
    if (acc == 12345.678) out[0] = acc;
}
__global__ void k_store8(double* __restrict__ p, size_t n) {
    for (size_t i = blockIdx.x * 256 + threadIdx.x; i < n; i += (size_t)gridDim.x * 256) p[i] = (double)i;
}
__global__ void k_slots(const double* __restrict__ P, int nslots, int S, int n, double* out) {
    const int k = threadIdx.x & 15, grp = threadIdx.x >> 4;
    const int i = min(blockIdx.x * 16 + grp, n - 1);
    double acc = 0.;
    for (int s0 = k; s0 < nslots; s0 += 64)
        for (int u = 0; u < 4; ++u)
            for (int c = 0; c < 3; ++c) {
                const int sl = s0 + 16 * u;
                if (sl < nslots) acc += P[(size_t)sl * 3 * S + (size_t)c * S + i];
            }
    if (acc == 12345.678) out[0] = acc;
}
__global__ void k_state(const double* __restrict__ R, const double* __restrict__ V, const double* __restrict__ T,
                        const double* __restrict__ psi, int S, int n, double* out) {
    const int k = threadIdx.x & 15, grp = threadIdx.x >> 4;
    const int i = min(blockIdx.x * 16 + grp, n - 1);
    const int c = k < 3 ? k : 0;
    double acc = R[(size_t)c * S + i] + V[(size_t)c * S + i] + T[i];
    if (k < 12) acc += psi[(size_t)(2 * k) * S + i] + psi[(size_t)(2 * k + 1) * S + i];
    if (acc == 12345.678) out[0] = acc;
}

int main() {
    const size_t big = (size_t)512 << 20, n64 = ((size_t)64 << 20) / 8;
    double *scrub, *buf, *out;
    CHK(hipMalloc(&scrub, big));
    CHK(hipMalloc(&buf, (size_t)64 << 20));
    CHK(hipMalloc(&out, 64));
    CHK(hipMemset(buf, 0, (size_t)64 << 20));
    const int N = 3573, S = 3584, nslots = 56;
    double* P;
    CHK(hipMalloc(&P, (size_t)nslots * 3 * S * 8));
    CHK(hipMemset(P, 0, (size_t)nslots * 3 * S * 8));
    double *R, *V, *T, *psi;
    CHK(hipMalloc(&R, 3 * S * 8)); CHK(hipMalloc(&V, 3 * S * 8)); CHK(hipMalloc(&T, S * 8)); CHK(hipMalloc(&psi, 24 * S * 8));
    CHK(hipMemset(R, 0, 3 * S * 8)); CHK(hipMemset(V, 0, 3 * S * 8)); CHK(hipMemset(T, 0, S * 8)); CHK(hipMemset(psi, 0, 24 * S * 8));
    const int ngrp = (N + 15) / 16;
    for (int rep = 0; rep < 5; ++rep) {
        hipLaunchKernelGGL(k_store8, dim3(4096), dim3(256), 0, 0, scrub, big / 8);   // scrub L2 / MALL
        hipLaunchKernelGGL(k_stream16, dim3(2048), dim3(256), 0, 0, (const double2*)buf, n64 / 2, out);
        hipLaunchKernelGGL(k_store8, dim3(4096), dim3(256), 0, 0, scrub, big / 8);
        hipLaunchKernelGGL(k_stream8, dim3(2048), dim3(256), 0, 0, buf, n64, out);
        hipLaunchKernelGGL(k_store8, dim3(4096), dim3(256), 0, 0, scrub, big / 8);
        hipLaunchKernelGGL(k_slots, dim3(ngrp), dim3(256), 0, 0, P, nslots, S, N, out);
        hipLaunchKernelGGL(k_store8, dim3(4096), dim3(256), 0, 0, scrub, big / 8);
        hipLaunchKernelGGL(k_state, dim3(ngrp), dim3(256), 0, 0, R, V, T, psi, S, N, out);
        hipLaunchKernelGGL(k_store8, dim3(2048), dim3(256), 0, 0, buf, n64);
    }
    CHK(hipDeviceSynchronize());
    // known bytes: slot lines = planes x lines covering ions [0, N) of each plane (S a multiple of 16)
    const double lines_per_plane = (double)((N + 15) / 16);
    printf("known bytes: k_stream16 %zu, k_stream8 %zu, k_store8(buf) %zu, k_slots %.0f, k_state %.0f\n",
           (size_t)64 << 20, (size_t)64 << 20, (size_t)64 << 20, nslots * 3 * lines_per_plane * 128.,
           (3 + 3 + 1 + 24) * lines_per_plane * 128.);
    return 0;
}
