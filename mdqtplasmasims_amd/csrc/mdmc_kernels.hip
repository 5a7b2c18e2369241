// gfx950 kernels of the Monte-Carlo + MD analytics program:
// MonteCarloFollowedByMDAndTempAnisotropy.cpp ("MCMD") — Metropolis anneal, velocity-Verlet
// updates, pair potentials, g(r), velocity autocorrelations, tagged moments, temperatures.
// The pair forces of the MD steps are the Newton-3 tile kernel of mdqt_forces.hip (the same
// Yukawa law: calcAIJ :161-169 = (1/r + kappa) e^{-kappa r} / r^2 with lDeb = 1/kappa).
//
// Built with -ffp-contract=off and no fast-math: expressions keep the reference's operation
// order, so the only device/host differences left are libm ulps (exp) and reduction orders.
#include "mdqt_internal.hpp"

#include <math.h>

namespace mdqt {

// ------------------------------------------------------------------------------------------
// The reference's RNG on the device: std::mt19937 (MCMD:53) and libstdc++'s
// generate_canonical<double, 53> behind uniform_real_distribution<double>(0, 1) (MCMD:54):
// u = (g1 + g2 2^32) / 2^64, clamped below 1.  Single-lane use only (state in LDS).
// ------------------------------------------------------------------------------------------
__device__ void mt_twist(uint32_t* x) {
    for (int k = 0; k < 624; ++k) {
        const uint32_t y = (x[k] & 0x80000000u) | (x[k + 1 < 624 ? k + 1 : 0] & 0x7fffffffu);
        const int m = k + 397 < 624 ? k + 397 : k + 397 - 624;
        x[k] = x[m] ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
    }
}
__device__ uint32_t mt_next(uint32_t* x, int& p) {
    if (p >= 624) { mt_twist(x); p = 0; }
    uint32_t z = x[p++];
    z ^= z >> 11;
    z ^= (z << 7) & 0x9d2c5680u;
    z ^= (z << 15) & 0xefc60000u;
    z ^= z >> 18;
    return z;
}
__device__ double mt_uniform(uint32_t* x, int& p) {
    double sum = (double)mt_next(x, p);
    sum = sum + (double)mt_next(x, p) * 4294967296.0;
    const double r = sum / 18446744073709551616.0;
    return r >= 1.0 ? 0x1.fffffffffffffp-1 : r;
}

__device__ __forceinline__ double mic_div(double d, double L) { return d - L * round(d / L); }   // :228-230
__device__ __forceinline__ double mc_uij(double r, double kappa, double rCut) {                 // calcUIJ :153-159
    if (r < rCut) return exp(-1 * kappa * r) / r;
    return 0.;
}
__device__ __forceinline__ double wave_sum(double v) {      // butterfly: every lane holds the same sum
    for (int o = 32; o > 0; o >>= 1) v = v + __shfl_xor(v, o);
    return v;
}

// ------------------------------------------------------------------------------------------
// calculatePotentialEnergyForParticles (:207-245): U[i] = sum_{j != i} u(r_ij), j ascending
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_particle_potentials(const double* __restrict__ R, int N, int S, double L,
                                                             double kappa, double rCut, double* __restrict__ U) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    const double cx = R[i], cy = R[S + i], cz = R[2 * S + i];
    double u = 0.;
    for (int j = 0; j < N; ++j) {
        const double xd = mic_div(cx - R[j], L), yd = mic_div(cy - R[S + j], L), zd = mic_div(cz - R[2 * S + j], L);
        const double d = sqrt(xd * xd + yd * yd + zd * zd);
        if (j != i) u += mc_uij(d, kappa, rCut);
    }
    U[i] = u;
}

// ------------------------------------------------------------------------------------------
// Metropolis anneal (MonteCarloStep :315-382, changePotentialEnergy :249-313): one workgroup
// runs the steps in sequence; lane 0 draws (mt19937 in LDS), all 1024 threads evaluate the
// O(N) energy change, lane 0 accepts or rejects.  U, the candidate U' and R stay in HBM/L2.
// ------------------------------------------------------------------------------------------
constexpr int MCT = 1024;

__global__ __launch_bounds__(MCT) void k_monte_carlo(MCArgs a) {
    __shared__ uint32_t smt[624];
    __shared__ int s_p, s_P, s_acc;
    __shared__ double s_d[3], s_tot;
    __shared__ double s_part[2][MCT / 64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    for (int k = tid; k < 624; k += MCT) smt[k] = a.mt[k];
    if (tid == 0) s_p = (int)a.mt[624];
    __syncthreads();
    const int N = a.N, S = a.S;
    double* X = a.R;
    double* Y = a.R + S;
    double* Z = a.R + 2 * S;
    const double L = a.L;
    unsigned long long acc = 0;
    for (int step = 0; step < a.nsteps; ++step) {
        if (tid == 0) {                                            // :325-334
            int p = s_p, P;
            double rx, ry, rz;
            for (;;) {
                const double randPart = mt_uniform(smt, p);
                P = (int)floor(randPart * N);
                rx = a.maxRStep * (2 * mt_uniform(smt, p) - 1);
                ry = a.maxRStep * (2 * mt_uniform(smt, p) - 1);
                rz = a.maxRStep * (2 * mt_uniform(smt, p) - 1);
                if (rx * rx + ry * ry + rz * rz < a.maxRStep * a.maxRStep) break;
            }
            s_p = p; s_P = P; s_d[0] = rx; s_d[1] = ry; s_d[2] = rz;
        }
        __syncthreads();
        const int P = s_P;
        const double ox = X[P], oy = Y[P], oz = Z[P];
        double nx = ox + s_d[0], ny = oy + s_d[1], nz = oz + s_d[2];   // :262-271
        if (nx < 0) nx += L;
        if (nx > L) nx -= L;
        if (ny < 0) ny += L;
        if (ny > L) ny -= L;
        if (nz < 0) nz += L;
        if (nz > L) nz -= L;
        double tot = 0., dsum = 0.;
        for (int j = tid; j < N; j += MCT) {                       // :273-310
            if (j == P) continue;
            const double cx = X[j], cy = Y[j], cz = Z[j];
            const double xn = mic_div(nx - cx, L), yn = mic_div(ny - cy, L), zn = mic_div(nz - cz, L);
            const double xo = mic_div(ox - cx, L), yo = mic_div(oy - cy, L), zo = mic_div(oz - cz, L);
            const double dO = sqrt(xo * xo + yo * yo + zo * zo);
            const double dN = sqrt(xn * xn + yn * yn + zn * zn);
            const double uN = mc_uij(dN, a.kappa, a.rCut), uO = mc_uij(dO, a.kappa, a.rCut);
            tot = tot + uN;
            const double Uj = a.U[j];
            const double Un = Uj + (uN - uO);                      // U[j] += (UijNew - UijOld)
            a.D[j] = Un;
            dsum = dsum + (Un - Uj);
        }
        tot = wave_sum(tot);
        dsum = wave_sum(dsum);
        if (lane == 0) { s_part[0][w] = tot; s_part[1][w] = dsum; }
        __syncthreads();
        if (tid == 0) {
            double T = 0., Dd = 0.;
            for (int q = 0; q < MCT / 64; ++q) { T = T + s_part[0][q]; Dd = Dd + s_part[1][q]; }
            const double dE = Dd + (T - a.U[P]);                  // sum_i U[i] - oldU[i] (:341-345)
            bool good = dE < 0;                                    // :347
            if (!good) {                                           // :353-360
                int p = s_p;
                const double dice = mt_uniform(smt, p);
                s_p = p;
                good = dice < exp(-(dE / 2) * a.Gamma);
            }
            s_acc = good;
            s_tot = T;
            if (good) { X[P] = nx; Y[P] = ny; Z[P] = nz; }         // :363-376
        }
        __syncthreads();
        if (s_acc) {
            for (int j = tid; j < N; j += MCT) a.U[j] = (j == P) ? s_tot : a.D[j];   // U[NPart] = totalU (:312)
            if (tid == 0) ++acc;
        }
        __syncthreads();
    }
    for (int k = tid; k < 624; k += MCT) a.mt[k] = smt[k];
    if (tid == 0) { a.mt[624] = (uint32_t)s_p; *a.accepted += acc; }
}

// ------------------------------------------------------------------------------------------
// LDS-resident Metropolis for N <= NPT * 1024 (N = 4096: NPT = 4).  Positions live in LDS
// (24 N bytes), each thread keeps U[j] and the candidate U'[j] of its NPT particles in
// registers, a step costs two barriers, and the minimum image is the division-free form
// d - L s, s = (d >= micT) - (d <= -micT) (= round(d/L) exactly for |d| < 1.25 L; positions
// stay in [0, L], MCMD:262-271).  The mt19937 state is double-buffered in LDS: the last wave
// twists the next block of 624 words (three dependency phases, 64 lanes) while the step's
// energies are summed, so lane 0 never runs the serial twist unless a step draws > 624 words.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ uint32_t mt_mix(uint32_t a, uint32_t b, uint32_t m) {
    const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
    return m ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
}
__device__ __forceinline__ void lds_wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_SEQ_CST, "wavefront");
    __builtin_amdgcn_s_waitcnt(0xc07f);     // lgkmcnt(0): the wave's LDS writes have landed
    __builtin_amdgcn_wave_barrier();
}
// Y = twist(X) by one wave (X untouched)
__device__ void mt_twist_wave(const uint32_t* X, uint32_t* Y, int lane) {
    for (int k = lane; k < 227; k += 64) Y[k] = mt_mix(X[k], X[k + 1], X[k + 397]);
    lds_wave_sync();
    for (int k = 227 + lane; k < 454; k += 64) Y[k] = mt_mix(X[k], X[k + 1], Y[k - 227]);
    lds_wave_sync();
    for (int k = 454 + lane; k < 623; k += 64) Y[k] = mt_mix(X[k], X[k + 1], Y[k - 227]);
    lds_wave_sync();
    if (lane == 0) Y[623] = mt_mix(X[623], Y[0], Y[396]);
    lds_wave_sync();
}
struct MtLds {
    uint32_t w[2][624];
    int p, cur, ahead;      // position in w[cur]; ahead: w[cur ^ 1] == twist(w[cur])
};
struct MtPos {
    int p, cur, ahead;      // thread 0's register copy of the MtLds bookkeeping
};
__device__ __forceinline__ double mt_uniform_lds(MtLds& m, MtPos& r) {
    double r2[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
        if (r.p >= 624) {
            if (r.ahead) { r.cur ^= 1; r.ahead = 0; }
            else mt_twist(m.w[r.cur]);                        // > 624 words in one step: in place
            r.p = 0;
        }
        uint32_t z = m.w[r.cur][r.p++];
        z ^= z >> 11;
        z ^= (z << 7) & 0x9d2c5680u;
        z ^= (z << 15) & 0xefc60000u;
        z ^= z >> 18;
        r2[h] = (double)z;
    }
    const double u = (r2[0] + r2[1] * 4294967296.0) / 18446744073709551616.0;
    return u >= 1.0 ? 0x1.fffffffffffffp-1 : u;
}
__device__ __forceinline__ uint32_t mt_temper(uint32_t z) {
    z ^= z >> 11;
    z ^= (z << 7) & 0x9d2c5680u;
    z ^= (z << 15) & 0xefc60000u;
    z ^= z >> 18;
    return z;
}
__device__ __forceinline__ double mt_canonical(uint32_t g1, uint32_t g2) {   // generate_canonical<double, 53>
    const double u = ((double)g1 + (double)g2 * 4294967296.0) / 18446744073709551616.0;
    return u >= 1.0 ? 0x1.fffffffffffffp-1 : u;
}
// the four uniforms of one proposal attempt (MCMD:326-331): the 8 words are read with independent
// LDS loads (one latency instead of eight) when they lie in the current buffer
__device__ __forceinline__ void mt_uniform4_lds(MtLds& m, MtPos& r, double* u) {
    if (r.p + 8 <= 624) {
        const uint32_t* src = m.w[r.cur] + r.p;
        uint32_t g[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) g[k] = src[k];
        r.p += 8;
#pragma unroll
        for (int k = 0; k < 4; ++k) u[k] = mt_canonical(mt_temper(g[2 * k]), mt_temper(g[2 * k + 1]));
        return;
    }
#pragma unroll
    for (int k = 0; k < 4; ++k) u[k] = mt_uniform_lds(m, r);
}
__device__ __forceinline__ double mic_t(double d, double L, double T) {
    const double s = (double)(d >= T) - (double)(d <= -T);
    return d - L * s;
}

// pair energy u(r) of one separation (calcUIJ :153-159) with the reference's pair set: the exact
// division-free minimum image and r2 as :292-293; the lattice start puts pairs exactly on the
// cutoff, so FAST tests r2 < rc2 (= sqrt(r2) < rCut) and only then takes the value through
// rsq3 and exp_neg (a few ulp, no division or library call).  Otherwise the
// reference's operations (sqrt, libm exp, division).
__device__ __forceinline__ double mic_c(double d, double L, double T) {   // = mic_t, 4 operations
    return (fabs(d) >= T) ? d - copysign(L, d) : d;
}
template <bool FAST>
__device__ __forceinline__ double mc_pair(double dx, double dy, double dz, const MCArgs& a) {
    dx = mic_c(dx, a.L, a.micT);
    dy = mic_c(dy, a.L, a.micT);
    dz = mic_c(dz, a.L, a.micT);
    const double r2 = dx * dx + dy * dy + dz * dz;                    // :292-293
    if (FAST) {
        const double ri = rsq3(r2);
        const double u = exp_neg(-a.kappa * (r2 * ri)) * ri;
        return r2 < a.rc2 ? u : 0.;                                    // = sqrt(r2) < rCut
    }
    return mc_uij(sqrt(r2), a.kappa, a.rCut);
}

template <int NPT, bool FAST>
__global__ __launch_bounds__(MCT) void k_monte_carlo_lds(MCArgs a) {
    extern __shared__ double sR[];                   // [3][N]
    __shared__ MtLds mt;
    __shared__ int s_P, s_acc;
    __shared__ double s_d[3], s_tot, s_UP;
    __shared__ double s_part[2][MCT / 64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    const int N = a.N, S = a.S;
    const double L = a.L;
    double* X = sR;
    double* Y = sR + N;
    double* Z = sR + 2 * N;
    for (int k = tid; k < N; k += MCT) { X[k] = a.R[k]; Y[k] = a.R[S + k]; Z[k] = a.R[2 * S + k]; }
    for (int k = tid; k < 624; k += MCT) mt.w[0][k] = a.mt[k];
    double U[NPT], Un[NPT];
#pragma unroll
    for (int q = 0; q < NPT; ++q) {
        const int j = tid + q * MCT;
        U[q] = j < N ? a.U[j] : 0.;
        Un[q] = U[q];
    }
    if (tid == 0) { mt.p = (int)a.mt[624]; mt.cur = 0; mt.ahead = 0; s_acc = 0; }
    __syncthreads();
    if (w == MCT / 64 - 1) {
        mt_twist_wave(mt.w[0], mt.w[1], lane);
        if (lane == 0) mt.ahead = 1;
    }
    __syncthreads();
    unsigned long long acc = 0;
    auto draw = [&](MtPos& r) {                                      // MCMD:325-334 (tid 0)
        int P;
        double rx, ry, rz;
        for (;;) {
            double u[4];
            mt_uniform4_lds(mt, r, u);
            const double randPart = u[0];
            P = (int)floor(randPart * N);
            rx = a.maxRStep * (2 * u[1] - 1);
            ry = a.maxRStep * (2 * u[2] - 1);
            rz = a.maxRStep * (2 * u[3] - 1);
            if (rx * rx + ry * ry + rz * rz < a.maxRStep * a.maxRStep) break;
        }
        s_P = P; s_d[0] = rx; s_d[1] = ry; s_d[2] = rz;
    };
    if (tid == 0 && a.nsteps > 0) {
        MtPos r{mt.p, mt.cur, mt.ahead};
        draw(r);
        mt.p = r.p; mt.cur = r.cur; mt.ahead = r.ahead;
    }
    __syncthreads();
    int prevP = -1;
    double nx = 0., ny = 0., nz = 0.;
    for (int step = 0; step < a.nsteps; ++step) {
        // ---- all threads: the previous step's acceptance, then the energy change (:249-313)
        if (s_acc) {
            const double tt = s_tot;
#pragma unroll
            for (int q = 0; q < NPT; ++q) U[q] = (tid + q * MCT == prevP) ? tt : Un[q];   // U[NPart] = totalU
        }
        const int P = s_P;
        const double ox = X[P], oy = Y[P], oz = Z[P];
        nx = ox + s_d[0]; ny = oy + s_d[1]; nz = oz + s_d[2];          // :262-271
        if (nx < 0) nx += L;
        if (nx > L) nx -= L;
        if (ny < 0) ny += L;
        if (ny > L) ny -= L;
        if (nz < 0) nz += L;
        if (nz > L) nz -= L;
        double tot = 0., dsum = 0.;
#pragma unroll
        for (int q = 0; q < NPT; ++q) {
            const int j = tid + q * MCT;
            Un[q] = U[q];
            if (j >= N) continue;
            if (j == P) { s_UP = U[q]; continue; }
            const double cx = X[j], cy = Y[j], cz = Z[j];
            const double uN = mc_pair<FAST>(nx - cx, ny - cy, nz - cz, a);
            const double uO = mc_pair<FAST>(ox - cx, oy - cy, oz - cz, a);
            tot = tot + uN;
            Un[q] = U[q] + (uN - uO);                                   // U[j] += (UijNew - UijOld)
            dsum = dsum + (Un[q] - U[q]);
        }
        tot = wave_sum(tot);
        dsum = wave_sum(dsum);
        if (lane == 0) { s_part[0][w] = tot; s_part[1][w] = dsum; }
        if (w == MCT / 64 - 1 && !mt.ahead) {                           // twist ahead off the critical path
            mt_twist_wave(mt.w[mt.cur], mt.w[mt.cur ^ 1], lane);
            if (lane == 0) mt.ahead = 1;
        }
        prevP = P;
        __syncthreads();
        // ---- thread 0: accept / reject (:341-381), then the next step's draws
        if (tid == 0) {
            MtPos r{mt.p, mt.cur, mt.ahead};
            double t16[MCT / 64], d16[MCT / 64];                           // fixed-shape trees: depth 4
#pragma unroll
            for (int q = 0; q < MCT / 64; ++q) { t16[q] = s_part[0][q]; d16[q] = s_part[1][q]; }
#pragma unroll
            for (int h = MCT / 128; h >= 1; h >>= 1)
#pragma unroll
                for (int q = 0; q < h; ++q) { t16[q] = t16[2 * q] + t16[2 * q + 1]; d16[q] = d16[2 * q] + d16[2 * q + 1]; }
            const double Tt = t16[0], Dd = d16[0];
            const double dE = Dd + (Tt - s_UP);
            bool good = dE < 0;
            if (!good) {                                                     // :353-360
                const double dice = mt_uniform_lds(mt, r);
                good = dice < (FAST ? exp_neg(-(dE / 2) * a.Gamma) : exp(-(dE / 2) * a.Gamma));
            }
            s_acc = good;
            s_tot = Tt;
            if (good) { X[P] = nx; Y[P] = ny; Z[P] = nz; ++acc; }
            if (step + 1 < a.nsteps) draw(r);
            mt.p = r.p; mt.cur = r.cur; mt.ahead = r.ahead;
        }
        __syncthreads();
    }
    if (s_acc) {
        const double tt = s_tot;
#pragma unroll
        for (int q = 0; q < NPT; ++q) U[q] = (tid + q * MCT == prevP) ? tt : Un[q];
    }
#pragma unroll
    for (int q = 0; q < NPT; ++q) {
        const int j = tid + q * MCT;
        if (j < N) a.U[j] = U[q];
    }
    for (int k = tid; k < N; k += MCT) { a.R[k] = X[k]; a.R[S + k] = Y[k]; a.R[2 * S + k] = Z[k]; }
    for (int k = tid; k < 624; k += MCT) a.mt[k] = mt.w[mt.cur][k];
    if (tid == 0) { a.mt[624] = (uint32_t)mt.p; *a.accepted += acc; }
}

// ------------------------------------------------------------------------------------------
// velocity Verlet (MDStep :504-511).  k_vv_positions is stepPositions :452-467 (R -> Rn).  After
// the Newton-3 force kernel, k_vv_step sums the force slots (canonical order) into a(t + dt),
// runs stepVelocities :469-502 (Verlet update + laser force) and pre-advances the positions of
// the next MDStep, r + dt v + dt^2/2 a with the box wrap, into Rn: the same expression on the same
// values stepPositions would read, so a step is two launches.  k_collide then overwrites the
// collided particles of the step from the host-drawn list (and redoes their Rn).
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ double step_pos(double r, double v, double a, double dt, double L) {   // :455-464
    r = r + dt * v + dt * dt / 2 * a;
    if (r < 0) r += L;
    if (r > L) r -= L;
    return r;
}

__global__ __launch_bounds__(256) void k_vv_positions(const double* __restrict__ R, const double* __restrict__ V,
                                                      const double* __restrict__ A, double* __restrict__ Rn,
                                                      int N, int S, double dt, double L) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const size_t k = (size_t)c * S + i;
        Rn[k] = step_pos(R[k], V[k], A[k], dt, L);
    }
}

__device__ __forceinline__ void laser_kick(const VVArgs& a, double* v) {      // :488-498
    if (a.oneAxis) {
        v[0] += v[0] * a.dt * 1.234 * a.p6 * a.beta / a.sqrtn;
    } else {
        v[0] += v[0] * a.dt * 1.234 * a.p6 * a.beta / a.sqrtn / 2;
        v[1] += v[1] * a.dt * 1.234 * a.p6 * a.beta / a.sqrtn / 4 * (-1);
        v[2] += v[2] * a.dt * 1.234 * a.p6 * a.beta / a.sqrtn / 4 * (-1);
    }
}

__device__ __forceinline__ double laser_term(const VVArgs& a, int c, double v) {   // :488-498, component c
    if (a.oneAxis) return c == 0 ? v + v * a.dt * 1.234 * a.p6 * a.beta / a.sqrtn : v;
    if (c == 0) return v + v * a.dt * 1.234 * a.p6 * a.beta / a.sqrtn / 2;
    return v + v * a.dt * 1.234 * a.p6 * a.beta / a.sqrtn / 4 * (-1);
}

// workgroup = 64 particles x one component; wave q sums the slots q, q + 8, q + 16, ... of its
// 64 particles (coalesced rows) = seg_sum's accumulator a[q], and wave 0 combines the eight in
// seg_sum's tree: bit-identical to seg_sum, with 8x the loads in flight
__global__ __launch_bounds__(512) void k_vv_step(VVArgs a) {
    __shared__ double acc[8][64];
    const int lane = threadIdx.x & 63, q = threadIdx.x >> 6;
    const int i = blockIdx.x * 64 + lane;
    const int c = blockIdx.y;
    const size_t k = (size_t)c * a.S + i;
    const size_t stride = (size_t)3 * a.S;
    double sq = 0.;
    if (i < a.N)
        for (int sl = q; sl < a.nslots; sl += 8) sq += a.slots[(size_t)sl * stride + k];
    acc[q][lane] = sq;
    __syncthreads();
    if (q != 0 || i >= a.N) return;
    const double an = ((acc[0][lane] + acc[1][lane]) + (acc[2][lane] + acc[3][lane])) +
                      ((acc[4][lane] + acc[5][lane]) + (acc[6][lane] + acc[7][lane]));
    double v = a.V[k] + a.dt / 2 * (a.A[k] + an);                    // :484-486 (oldA + A)
    if (a.laser) v = laser_term(a, c, v);
    a.V[k] = v;
    a.A[k] = an;
    a.Rn[k] = step_pos(a.R[k], v, an, a.dt, a.L);
}

// the collided particles of the step (:477-482): V = the host-drawn Maxwellian, then the laser term
__global__ __launch_bounds__(64) void k_collide(VVArgs a) {
    const int h = blockIdx.x * 64 + threadIdx.x;
    if (h >= a.nhits) return;
    const double* e = a.hits + 4 * (size_t)h;
    const int i = (int)e[0];
    double v[3] = {e[1], e[2], e[3]};
    if (a.laser) laser_kick(a, v);
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const size_t k = (size_t)c * a.S + i;
        a.V[k] = v[c];
        a.Rn[k] = step_pos(a.R[k], v[c], a.A[k], a.dt, a.L);
    }
}

// ------------------------------------------------------------------------------------------
// g(r) histogram (recordPairPairCorr :591-622): block per particle i, integer bin counts in
// LDS then global (exact, order-free)
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_pair_hist(const double* __restrict__ R, int N, int S, double L, double step,
                                                   int nbins, unsigned* __restrict__ hist) {
    extern __shared__ unsigned hsh[];
    for (int b = threadIdx.x; b < nbins; b += 256) hsh[b] = 0;
    __syncthreads();
    const int i = blockIdx.x;
    const double cx = R[i], cy = R[S + i], cz = R[2 * S + i];
    for (int j = threadIdx.x; j < N; j += 256) {
        if (j == i) continue;
        const double xd = mic_div(cx - R[j], L), yd = mic_div(cy - R[S + j], L), zd = mic_div(cz - R[2 * S + j], L);
        const double d = sqrt(xd * xd + yd * yd + zd * zd);
        const int bin = (int)floor((double)(int)(d / step));       // :615
        if (bin < nbins) atomicAdd(&hsh[bin], 1u);                 // :616-618
    }
    __syncthreads();
    for (int b = threadIdx.x; b < nbins; b += 256)
        if (hsh[b]) atomicAdd(&hist[b], hsh[b]);
}

// ------------------------------------------------------------------------------------------
// velocity autocorrelations (:655-807) over vStore [3][N][T]: block b takes particles
// [b*pg, (b+1)*pg), their three series staged in LDS one particle at a time; thread t owns the
// lags td = t, t + 256, ...; partial sums per block in fixed order, then k_autocorr_reduce.
// ------------------------------------------------------------------------------------------
constexpr int ACT = 256;
constexpr int ACSLOTS = 16;                                        // T <= 4096

__global__ __launch_bounds__(ACT) void k_autocorr(const double* __restrict__ vs, int N, int T, int pg, double c2,
                                                  double c4, double* __restrict__ part) {
    extern __shared__ double sv[];                                 // [3][T]
    const int t0 = threadIdx.x;
    double acc[4][ACSLOTS];
#pragma unroll
    for (int f = 0; f < 4; ++f)
#pragma unroll
        for (int s = 0; s < ACSLOTS; ++s) acc[f][s] = 0.;
    const int i0 = blockIdx.x * pg, i1 = min(N, i0 + pg);
    for (int i = i0; i < i1; ++i) {
        __syncthreads();
        for (int k = t0; k < 3 * T; k += ACT) {
            const int c = k / T, t = k - c * T;
            sv[k] = vs[((size_t)c * N + i) * T + t];
        }
        __syncthreads();
        const double* x = sv;
        const double* y = sv + T;
        const double* z = sv + 2 * T;
#pragma unroll
        for (int s = 0; s < ACSLOTS; ++s) {
            const int td = t0 + s * ACT;
            if (td >= T) break;
            double f0 = 0., f1 = 0., f2 = 0., f3 = 0.;
            for (int j = 0; j < T - td; ++j) {
                const double x0 = x[j], x1 = x[j + td], y0 = y[j], y1 = y[j + td], z0 = z[j], z1 = z[j + td];
                f0 = f0 + (x0 * x1 + y0 * y1 + z0 * z1);                                   // :672
                const double px = (x0 * x0) * (x1 * x1), py = (y0 * y0) * (y1 * y1), pz = (z0 * z0) * (z1 * z1);
                f1 = f1 + (px + py + pz - c2);                                             // :710
                f2 = f2 + (px * x0 * x1 + py * y0 * y1 + pz * z0 * z1);                    // :748
                f3 = f3 + (px * (x0 * x0) * (x1 * x1) + py * (y0 * y0) * (y1 * y1) +
                           pz * (z0 * z0) * (z1 * z1) - c4);                               // :785
            }
            acc[0][s] += f0; acc[1][s] += f1; acc[2][s] += f2; acc[3][s] += f3;
        }
    }
#pragma unroll
    for (int s = 0; s < ACSLOTS; ++s) {
        const int td = t0 + s * ACT;
        if (td >= T) break;
#pragma unroll
        for (int f = 0; f < 4; ++f) part[((size_t)blockIdx.x * 4 + f) * T + td] = acc[f][s];
    }
}

__global__ __launch_bounds__(256) void k_autocorr_reduce(const double* __restrict__ part, int nblk, int N, int T,
                                                         double* __restrict__ out) {
    const int k = blockIdx.x * 256 + threadIdx.x;                  // f * T + td
    if (k >= 4 * T) return;
    const int td = k % T;
    double s = 0.;
    for (int b = 0; b < nblk; ++b) s = s + part[(size_t)b * 4 * T + k];
    out[k] = s / (double)(unsigned)(N * (T - td));                 // / (N*(numVelAutoCorrsSteps - tDiff))
}

// ------------------------------------------------------------------------------------------
// block reductions of the per-step observables: temperatures (:525-546, :560-581) and the
// tagged-particle moments (:937-971); one workgroup, fixed order
// ------------------------------------------------------------------------------------------
constexpr int RBT = 1024;

__global__ __launch_bounds__(RBT) void k_temperatures(const double* __restrict__ V, int N, int S, double* __restrict__ out) {
    __shared__ double sp[4][RBT / 64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    double a = 0., x = 0., y = 0., z = 0.;
    for (int i = tid; i < N; i += RBT) {
        const double vx = V[i], vy = V[S + i], vz = V[2 * S + i];
        a = a + vx * vx; a = a + vy * vy; a = a + vz * vz;
        x = x + vx * vx; y = y + vy * vy; z = z + vz * vz;
    }
    a = wave_sum(a); x = wave_sum(x); y = wave_sum(y); z = wave_sum(z);
    if (lane == 0) { sp[0][w] = a; sp[1][w] = x; sp[2][w] = y; sp[3][w] = z; }
    __syncthreads();
    if (tid < 4) {
        double s = 0.;
        for (int q = 0; q < RBT / 64; ++q) s = s + sp[tid][q];
        out[tid] = s;
    }
}

__global__ __launch_bounds__(RBT) void k_tag_moments(const double* __restrict__ V, const int* __restrict__ tags, int N,
                                                     double* __restrict__ out) {
    __shared__ double sp[20][RBT / 64];
    const int tid = threadIdx.x, lane = tid & 63, w = tid >> 6;
    double m[20];
#pragma unroll
    for (int q = 0; q < 20; ++q) m[q] = 0.;
    for (int i = tid; i < N; i += RBT) {
        const double v = V[i];
        const double v2 = v * v, v3 = v * v * v, v4 = v * v * v * v;
#pragma unroll
        for (int t = 0; t < 4; ++t)
            if (tags[(size_t)t * N + i]) {
                m[5 * t] += v; m[5 * t + 1] += v2; m[5 * t + 2] += v3; m[5 * t + 3] += v4; m[5 * t + 4] += 1.;
            }
    }
#pragma unroll
    for (int q = 0; q < 20; ++q) {
        const double s = wave_sum(m[q]);
        if (lane == 0) sp[q][w] = s;
    }
    __syncthreads();
    if (tid < 20) {
        double s = 0.;
        for (int q = 0; q < RBT / 64; ++q) s = s + sp[tid][q];
        out[tid] = s;
    }
}

// recordVelsForAutocorrelations (:513-523): vStore[c][i][t] = V[c][i]
__global__ __launch_bounds__(256) void k_store_velocities(const double* __restrict__ V, int N, int S, int T, int t,
                                                          double* __restrict__ vs) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
#pragma unroll
    for (int c = 0; c < 3; ++c) vs[((size_t)c * N + i) * T + t] = V[(size_t)c * S + i];
}

// anisotropizeVelocities (:548-558)
__global__ __launch_bounds__(256) void k_anisotropize(double* __restrict__ V, int N, int S, double tpd) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= N) return;
    V[i] = sqrt(1 + tpd) * V[i];
    V[S + i] = sqrt(1 - tpd / 2) * V[S + i];
    V[2 * S + i] = sqrt(1 - tpd / 2) * V[2 * S + i];
}

// ------------------------------------------------------------------------------------------
// recordTaggedParticleMoments' distributions (QT tagging programs, QTT:1097-1124): bins
// vel_j = (j - 2000) 0.0025, P_c[j] = sum over tagged ions of exp(-V2 (vel_j - v_c)^2),
// V2 = 1/(2 0.002^2), / (6 sqrt(2 pi 0.002^2)).  Workgroup = 256 bins x one chunk of ions (LDS
// staged, ascending); the chunk partials are summed in chunk order by k_tagged_kde_reduce.
// ------------------------------------------------------------------------------------------
constexpr int TKDE_CHUNK = 256;

__global__ __launch_bounds__(256) void k_tagged_kde(const double* __restrict__ V, const int* __restrict__ tags, int N,
                                                    int S, int bin0, double* __restrict__ part) {
    __shared__ double sv[3][TKDE_CHUNK];
    __shared__ int st[TKDE_CHUNK];
    const int j = blockIdx.x * 256 + threadIdx.x;
    const int i0 = blockIdx.y * TKDE_CHUNK;
    const int i = i0 + threadIdx.x;
    if (i < N) {
        sv[0][threadIdx.x] = V[i]; sv[1][threadIdx.x] = V[S + i]; sv[2][threadIdx.x] = V[2 * S + i];
        st[threadIdx.x] = tags[i];
    } else {
        st[threadIdx.x] = 0;
    }
    __syncthreads();
    const double vel = (double)(j + bin0) * 0.0025;                 // QTT:250 (bin0 = -2000)
    const double V2 = kKdeV2;                                      // 1 / (2 * 0.002^2), QTT:1072
    double p[3] = {0., 0., 0.};
    const int m = min(TKDE_CHUNK, N - i0);
    for (int k = 0; k < m; ++k) {
        if (!st[k]) continue;                                      // uniform over the workgroup
        // a component whose term is exactly +0 on every bin of the wave (|vel - v| >= 0.0773:
        // V2 d^2 >= 746.9, below exp's underflow) adds exact zeros there and is skipped
#pragma unroll
        for (int c = 0; c < 3; ++c)
            if (__builtin_amdgcn_ballot_w64(!(fabs(vel - sv[c][k]) >= kKdeSkip)))
                p[c] += exp(-V2 * (vel - sv[c][k]) * (vel - sv[c][k]));   // :1100-1102
    }
    if (j < TKDE_BINS)
#pragma unroll
        for (int c = 0; c < 3; ++c) part[((size_t)blockIdx.y * 3 + c) * TKDE_BINS + j] = p[c];
}

__global__ __launch_bounds__(256) void k_tagged_kde_reduce(const double* __restrict__ part, int nch,
                                                           double* __restrict__ out) {
    const int k = blockIdx.x * 256 + threadIdx.x;                  // c * TKDE_BINS + j
    if (k >= 3 * TKDE_BINS) return;
    double s = 0.;
    for (int q = 0; q < nch; ++q) s = s + part[(size_t)q * 3 * TKDE_BINS + k];
    out[k] = s / (6.0 * sqrt(2 * M_PI * 0.002 * 0.002));            // :1121-1123
}

// ------------------------------------------------------------------------------------------
// launchers
// ------------------------------------------------------------------------------------------
hipError_t launch_particle_potentials(const double* R, int N, int S, double L, double kappa, double rCut, double* U,
                                      hipStream_t s) {
    if (N <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_particle_potentials, dim3((N + 255) / 256), dim3(256), 0, s, R, N, S, L, kappa, rCut, U);
    return hipGetLastError();
}
template <int NPT, bool FAST>
static hipError_t launch_mc_lds_v(const MCArgs& a, hipStream_t s) {
    const size_t lds = (size_t)3 * a.N * sizeof(double);
    hipError_t e = hipFuncSetAttribute((const void*)k_monte_carlo_lds<NPT, FAST>,
                                       hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL((k_monte_carlo_lds<NPT, FAST>), dim3(1), dim3(MCT), lds, s, a);
    return hipGetLastError();
}
template <int NPT>
static hipError_t launch_mc_lds(const MCArgs& a, hipStream_t s) {
    return a.fast ? launch_mc_lds_v<NPT, true>(a, s) : launch_mc_lds_v<NPT, false>(a, s);
}
hipError_t launch_monte_carlo(const MCArgs& a, hipStream_t s) {
    if (a.nsteps <= 0) return hipSuccess;
    const int npt = (a.N + MCT - 1) / MCT;
    switch (npt) {                                       // positions in LDS up to N = 6144 (144 KB)
        case 1: return launch_mc_lds<1>(a, s);
        case 2: return launch_mc_lds<2>(a, s);
        case 3: return launch_mc_lds<3>(a, s);
        case 4: return launch_mc_lds<4>(a, s);
        case 5: return launch_mc_lds<5>(a, s);
        case 6: return launch_mc_lds<6>(a, s);
        default: break;
    }
    hipLaunchKernelGGL(k_monte_carlo, dim3(1), dim3(MCT), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_vv_positions(const double* R, const double* V, const double* A, double* Rn, int N, int S, double dt,
                               double L, hipStream_t s) {
    if (N <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_vv_positions, dim3((N + 255) / 256), dim3(256), 0, s, R, V, A, Rn, N, S, dt, L);
    return hipGetLastError();
}
hipError_t launch_vv_velocities(const VVArgs& a, hipStream_t s) {
    if (a.N <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_vv_step, dim3((a.N + 63) / 64, 3), dim3(512), 0, s, a);
    if (a.nhits > 0) hipLaunchKernelGGL(k_collide, dim3((a.nhits + 63) / 64), dim3(64), 0, s, a);
    return hipGetLastError();
}
hipError_t launch_pair_hist(const double* R, int N, int S, double L, double step, int nbins, unsigned* hist,
                            hipStream_t s) {
    if (N <= 0 || nbins <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_pair_hist, dim3(N), dim3(256), nbins * sizeof(unsigned), s, R, N, S, L, step, nbins, hist);
    return hipGetLastError();
}
int autocorr_blocks(int N) { return N < 512 ? N : 512; }
hipError_t launch_autocorr(const double* vs, int N, int T, double c2, double c4, double* part, double* out,
                           hipStream_t s) {
    if (N <= 0 || T <= 0) return hipSuccess;
    if (T > ACT * ACSLOTS) return hipErrorInvalidValue;
    const int nblk = autocorr_blocks(N);
    const int pg = (N + nblk - 1) / nblk;
    const int used = (N + pg - 1) / pg;
    const size_t lds = (size_t)3 * T * sizeof(double);
    if (lds > 65536) {          // gfx950: up to 160 KB of LDS per workgroup on request
        const hipError_t e = hipFuncSetAttribute((const void*)k_autocorr, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        if (e != hipSuccess) return e;
    }
    hipLaunchKernelGGL(k_autocorr, dim3(used), dim3(ACT), lds, s, vs, N, T, pg, c2, c4, part);
    hipLaunchKernelGGL(k_autocorr_reduce, dim3((4 * T + 255) / 256), dim3(256), 0, s, part, used, N, T, out);
    return hipGetLastError();
}
hipError_t launch_temperatures(const double* V, int N, int S, double* out, hipStream_t s) {
    hipLaunchKernelGGL(k_temperatures, dim3(1), dim3(RBT), 0, s, V, N, S, out);
    return hipGetLastError();
}
hipError_t launch_tag_moments(const double* V, const int* tags, int N, double* out, hipStream_t s) {
    hipLaunchKernelGGL(k_tag_moments, dim3(1), dim3(RBT), 0, s, V, tags, N, out);
    return hipGetLastError();
}
hipError_t launch_store_velocities(const double* V, int N, int S, int T, int t, double* vs, hipStream_t s) {
    if (N <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_store_velocities, dim3((N + 255) / 256), dim3(256), 0, s, V, N, S, T, t, vs);
    return hipGetLastError();
}
hipError_t launch_anisotropize(double* V, int N, int S, double tpd, hipStream_t s) {
    if (N <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_anisotropize, dim3((N + 255) / 256), dim3(256), 0, s, V, N, S, tpd);
    return hipGetLastError();
}

// part must hold ceil(N / 256) x 3 x TKDE_BINS doubles, out 3 x TKDE_BINS
hipError_t launch_tagged_kde(const double* V, const int* tags, int N, int S, double* part, double* out, hipStream_t s,
                             int bin0) {
    if (N <= 0) return hipSuccess;
    const int nch = (N + TKDE_CHUNK - 1) / TKDE_CHUNK;
    hipLaunchKernelGGL(k_tagged_kde, dim3((TKDE_BINS + 255) / 256, nch), dim3(256), 0, s, V, tags, N, S, bin0, part);
    hipLaunchKernelGGL(k_tagged_kde_reduce, dim3((3 * TKDE_BINS + 255) / 256), dim3(256), 0, s, part, nch, out);
    return hipGetLastError();
}

}  // namespace mdqt
