// gfx950 kernels of the MDQT hot path (the force kernels are in mdqt_forces.hip).
//
//   k_substeps          n x (step(); qstep()) fused per ion, SpeedUp:356-430 + :438-717
//   k_substeps_lanes    the same, one ion per 16-lane group (lane = quantum state)
//   k_d48_resolve       drand48 in the reference's consumption order (rng_mode 0)
//   k_sum_vx / k_energy_sums / k_kde*   observables of output(), SpeedUp:917-1032
//
// Built with -ffp-contract=off and without fast-math: every floating-point expression keeps
// the reference's operation order (x86-64 g++ -O3 contracts nothing), so the only
// device/host differences left are libm ulps (exp, sin, cos).  See DESIGN.md §Parity.
#include "mdqt_device.hpp"

#include <math.h>

namespace mdqt {

// ------------------------------------------------------------------------------------------
// drand48 in the reference's consumption order (SpeedUp:486, :575-687).  X' = a X + c mod 2^48;
// 2^b steps compose to (jA[b], jC[b]).  One workgroup walks the ions in chunks of 1024: every
// ion of the chunk takes its u1 at (index + draws already shifted by earlier jumps); the first
// ion that jumps (u1 <= dp) takes 4 or 5 draws, which shifts everybody after it, and the walk
// restarts behind it.  Jumps are rare (dp ~ 1e-3), so a substep costs ~N/1024 + #jumps passes.
// ------------------------------------------------------------------------------------------
__device__ __forceinline__ unsigned long long lcg_adv(unsigned long long x, unsigned long long k,
                                                      const unsigned long long* jA,
                                                      const unsigned long long* jC) {
    for (int b = 0; k; ++b, k >>= 1)
        if (k & 1ull) x = (jA[b] * x + jC[b]) & 0xFFFFFFFFFFFFull;
    return x;
}

__global__ __launch_bounds__(1024) void k_d48_resolve(D48Args a) {
    __shared__ unsigned long long sA[48], sC[48];
    __shared__ int s_first[16];
    __shared__ int s_min, s_extra;
    const int tid = threadIdx.x, lane = tid & 63, wv = tid >> 6;
    if (tid < 48) { sA[tid] = a.jA[tid]; sC[tid] = a.jC[tid]; }
    __syncthreads();
    const QTConst& qc = a.qc;
    const int S = a.S, n = a.n;
    const unsigned long long X0 = *a.state;
    unsigned long long off = 0;
    int pos = 0;
    while (pos < n) {
        const int i = pos + tid;
        bool jmp = false;
        if (i < n) {
            const unsigned long long x = lcg_adv(X0, (unsigned long long)i + off + 1, sA, sC);
            const double u1 = ldexp((double)x, -48);
            double T[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const double re = a.psi[(size_t)(2 * (q + 2)) * S + i], im = a.psi[(size_t)(2 * (q + 2) + 1) * S + i];
                // exactly the dp of the substep kernel that consumes U (same jump decisions)
                if (a.fast == 2) T[q] = fma(re, re, im * im) * qc.hdPh[q];
                else if (a.fast == 1) T[q] = fma(re * qc.dP[q], re, (im * qc.dP[q]) * im);
                else T[q] = (re * qc.dP[q]) * re + (im * qc.dP[q]) * im;
            }
            const double dp = (a.fast == 2) ? (T[0] + T[1]) + (T[2] + T[3])          // mdqt_qtfast.hip
                                            : qc.h * (((T[0] + T[1]) + T[2]) + T[3]); // dp_of / row_sum_p
            jmp = !(u1 > dp);
            a.U[i] = u1;
        }
        const unsigned long long b = __ballot(jmp);
        if (lane == 0) s_first[wv] = b ? wv * 64 + __ffsll((long long)b) - 1 : 0x7fffffff;
        __syncthreads();
        if (tid == 0) {
            int m = 0x7fffffff;
            for (int w = 0; w < 16; ++w) m = min(m, s_first[w]);
            s_min = m;
            s_extra = 0;
        }
        __syncthreads();
        const int m = s_min;
        if (m == 0x7fffffff) {
            pos += 1024;
            __syncthreads();
            continue;
        }
        if (tid == m) {                               // the jumping ion: draws 2..4 (or 2..5)
            const unsigned long long k0 = (unsigned long long)i + off;
            const double rand2 = ldexp((double)lcg_adv(X0, k0 + 2, sA, sC), -48);
            const double randDOrS = ldexp((double)lcg_adv(X0, k0 + 3, sA, sC), -48);
            const double randDir = ldexp((double)lcg_adv(X0, k0 + 4, sA, sC), -48);
            double nrm[4];
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                const double re = a.psi[(size_t)(2 * (q + 2)) * S + i], im = a.psi[(size_t)(2 * (q + 2) + 1) * S + i];
                nrm[q] = re * re + im * im;
            }
            const double tot = nrm[0] + nrm[1] + nrm[2] + nrm[3];
            const double prob3 = nrm[0] / tot, prob4 = nrm[1] / tot, prob5 = nrm[2] / tot;
            const bool sDecay = !(randDOrS < qc.pD);
            bool need3;
            if (rand2 < prob3) need3 = !sDecay;
            else if (rand2 < prob3 + prob4) need3 = true;
            else if (rand2 < prob3 + prob4 + prob5) need3 = true;
            else need3 = !sDecay;
            const double rand3 = need3 ? ldexp((double)lcg_adv(X0, k0 + 5, sA, sC), -48) : 0.;
            a.U[(size_t)S + i] = rand2;
            a.U[(size_t)2 * S + i] = randDOrS;
            a.U[(size_t)3 * S + i] = randDir;
            a.U[(size_t)4 * S + i] = rand3;
            s_extra = need3 ? 4 : 3;
        }
        __syncthreads();
        off += (unsigned long long)s_extra;
        pos += m + 1;
        __syncthreads();
    }
    if (tid == 0) *a.state = lcg_adv(X0, (unsigned long long)n + off, sA, sC);
}

hipError_t launch_d48_resolve(const D48Args& a, hipStream_t s) {
    hipLaunchKernelGGL(k_d48_resolve, dim3(1), dim3(1024), 0, s, a);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Kernel 2: fused integrator + quantum-trajectory substeps, one thread per ion, the whole
// state (R, V, F, psi, tPart) held in registers across the nsub substeps of one launch
// (legal: between forces() calls no ion reads another ion).
// ------------------------------------------------------------------------------------------
// Re(h * y^H D y) with D = decayMatrix (diagonal, P levels only): SpeedUp:484-485, :530-531
template <bool F>
__device__ __forceinline__ double dp_of(const QTConst& qc, const cxd* y) {
    double v = decay_term<F>(y[2], qc.dP[0]);
    v = v + decay_term<F>(y[3], qc.dP[1]);
    v = v + decay_term<F>(y[4], qc.dP[2]);
    v = v + decay_term<F>(y[5], qc.dP[3]);
    return qc.h * v;
}

#define MS(i) cxd{qc.Mre[i], qc.Mim[i]}

// out = M y, M sparse (App. A); terms summed in ascending column order as the dense
// Armadillo product (exact zero terms dropped: they cannot change a non-zero sum).
template <bool F>
__device__ __forceinline__ void matvec(const QTConst& qc, const cxd* Md, const cxd& M49,
                                       const cxd& M58, const cxd& M85, const cxd& M94,
                                       const cxd* y, cxd* o) {
#define CM cmulT<F>
    o[0] = cadd(cadd(CM(Md[0], y[0]), CM(MS(0), y[3])), CM(MS(1), y[5]));
    o[1] = cadd(cadd(CM(Md[1], y[1]), CM(MS(2), y[2])), CM(MS(3), y[4]));
    o[2] = cadd(cadd(cadd(CM(MS(4), y[1]), CM(Md[2], y[2])), CM(MS(5), y[9])), CM(MS(6), y[11]));
    o[3] = cadd(cadd(cadd(CM(MS(7), y[0]), CM(Md[3], y[3])), CM(MS(8), y[8])), CM(MS(9), y[10]));
    o[4] = cadd(cadd(cadd(CM(MS(10), y[1]), CM(Md[4], y[4])), CM(MS(11), y[7])), CM(M49, y[9]));
    o[5] = cadd(cadd(cadd(CM(MS(12), y[0]), CM(Md[5], y[5])), CM(MS(13), y[6])), CM(M58, y[8]));
    o[6] = cadd(CM(MS(14), y[5]), CM(Md[6], y[6]));
    o[7] = cadd(CM(MS(15), y[4]), CM(Md[7], y[7]));
    o[8] = cadd(cadd(CM(MS(16), y[3]), CM(M85, y[5])), CM(Md[8], y[8]));
    o[9] = cadd(cadd(CM(MS(17), y[2]), CM(M94, y[4])), CM(Md[9], y[9]));
    o[10] = cadd(CM(MS(18), y[3]), CM(Md[10], y[10]));
    o[11] = cadd(CM(MS(19), y[2]), CM(Md[11], y[11]));
#undef CM
}

// One ion through qstep() (SpeedUp:478-712).  Returns the velocity kick.
template <bool F>
__device__ __forceinline__ double qstep_ion(const QTConst& qc, double eD, double vx,
                                            double& tPart, cxd* w, uint64_t gid, uint64_t q,
                                            const double* U, int S, int i) {
    const double velQuant = vx * qc.pv2q;                                  // :481-482
    tPart += qc.dtQ;                                                        // :483
    const double dp = dp_of<F>(qc, w);                                      // :484-485
    double u1, u2;
    draw_pair(qc, U, S, i, gid, q, 0, u1, u2);                              // :486
    double kick;
    if (u1 > dp) {                                                          // :487
        const double p23 = rho_im(w[1], w[2]), p14 = rho_im(w[0], w[3]);
        const double p25 = rho_im(w[1], w[4]), p16 = rho_im(w[0], w[5]);
        const double p96 = rho_im(w[8], w[5]), p105 = rho_im(w[9], w[4]);
        const double p114 = rho_im(w[10], w[3]), p123 = rho_im(w[11], w[2]);
        const double p76 = rho_im(w[6], w[5]), p85 = rho_im(w[7], w[4]);
        const double p94 = rho_im(w[8], w[3]), p103 = rho_im(w[9], w[2]);
        const double* gs = qc.gs;
        kick = qc.kickS * (p23 * gs[0] + p14 * gs[2] - p25 * gs[4] - p16 * gs[5]) * qc.dtQ * qc.gamToE +
               qc.kickD * (p96 * gs[8] + p105 * gs[11] + p114 * gs[14] + p123 * gs[17] - p76 * gs[6] -
                           p85 * gs[9] - p94 * gs[12] - p103 * gs[15]) * qc.dtQ * qc.gamToE;   // :503
        // Hamiltonian (:506-521) -> M = I - i h H (:525-526)
        const double vq = velQuant + eD;
        const double ER = -qc.det - velQuant - eD;                          // :506
        const double EL = -qc.det + velQuant + eD;                          // :507
        const double E67 = (-qc.det + qc.detDP + (1 - qc.kRat) * (velQuant + eD));
        const double E1011 = (-qc.det + qc.detDP + (qc.kRat - 1) * (velQuant + eD));
        const double E89 = (-qc.det + qc.detDP - velQuant - eD - qc.kRat * (velQuant + eD));
        const double phi = 2. * vq * (1 + qc.kRat) * tPart * qc.gamToE;   // :508
        double sn, cs;
        sincos_q<F>(phi, sn, cs);
        const double h = qc.h;
        cxd Md[NS];
        Md[0] = {1., -(h * 0.)};
        Md[1] = Md[0];
        Md[2] = {1. + h * qc.hdP[0], -(h * ER)};
        Md[3] = {1. + h * qc.hdP[1], -(h * ER)};
        Md[4] = {1. + h * qc.hdP[2], -(h * EL)};
        Md[5] = {1. + h * qc.hdP[3], -(h * EL)};
        Md[6] = {1., -(h * E67)};
        Md[7] = Md[6];
        Md[8] = {1., -(h * E89)};
        Md[9] = Md[8];
        Md[10] = {1., -(h * E1011)};
        Md[11] = Md[10];
        const double a8s = qc.a8 * sn, a8c = qc.a8 * cs, a11s = qc.a11 * sn, a11c = qc.a11 * cs;
        const cxd M85 = {-(h * a8s), h * a8c};
        const cxd M58 = {h * a8s, h * a8c};
        const cxd M94 = {-(h * a11s), h * a11c};
        const cxd M49 = {h * a11s, h * a11c};
        // k1..k4 (:530-567): k(y) = (M y / sqrt(1 - dp(y)) - y) / h
        cxd y[NS], ws[NS], acc[NS];
#pragma unroll
        for (int k = 0; k < NS; ++k) y[k] = w[k];
#pragma unroll
        for (int st = 0; st < 4; ++st) {
            const double pref = inv_sqrt_1m<F>(st == 0 ? dp : dp_of<F>(qc, y));
            matvec<F>(qc, Md, M49, M58, M85, M94, y, ws);
            const double step = (st == 2) ? h : qc.dtHalf;
#pragma unroll
            for (int k = 0; k < NS; ++k) {
                const cxd kk = {kstage<F>(qc.invh, pref, ws[k].re, y[k].re), kstage<F>(qc.invh, pref, ws[k].im, y[k].im)};
                if (st == 0) {
                    acc[k] = kk;
                } else if (st < 3) {
                    acc[k] = {axpy<F>(3., kk.re, acc[k].re), axpy<F>(3., kk.im, acc[k].im)};
                } else {
                    const cxd sum = {acc[k].re + kk.re, acc[k].im + kk.im};
                    w[k] = {axpy<F>(h, sum.re / 8, w[k].re), axpy<F>(h, sum.im / 8, w[k].im)};
                }
                if (st < 3) y[k] = {axpy<F>(step, kk.re, w[k].re), axpy<F>(step, kk.im, w[k].im)};
            }
        }
    } else {                                                                // :573-703
        tPart = 0;
        const double rand2 = u2;
        const double n3 = w[2].re * w[2].re + w[2].im * w[2].im;
        const double n4 = w[3].re * w[3].re + w[3].im * w[3].im;
        const double n5 = w[4].re * w[4].re + w[4].im * w[4].im;
        const double n6 = w[5].re * w[5].re + w[5].im * w[5].im;
        const double tot = n3 + n4 + n5 + n6;
        const double prob3 = n3 / tot, prob4 = n4 / tot, prob5 = n5 / tot;
        double randDOrS, randDir, rand3, dummy;
        draw_pair(qc, U, S, i, gid, q, 1, randDOrS, randDir);
        draw_pair(qc, U, S, i, gid, q, 2, rand3, dummy);
        (void)dummy;
        const bool sDecay = !(randDOrS < qc.pD);
        if (!sDecay) kick = (randDir < 0.5) ? qc.vKickDP : -qc.vKickDP;
        else kick = (randDir < 0.5) ? qc.vKick : -qc.vKick;
        int target;
        if (rand2 < prob3) {
            if (sDecay) target = 1;
            else target = (rand3 < qc.thD[0][0]) ? 11 : (rand3 < qc.thD[0][1]) ? 10 : 9;
        } else if (rand2 < prob3 + prob4) {
            if (sDecay) target = (rand3 < qc.thS3) ? 0 : 1;
            else target = (rand3 < qc.thD[1][0]) ? 10 : (rand3 < qc.thD[1][1]) ? 9 : 8;
        } else if (rand2 < prob3 + prob4 + prob5) {
            if (sDecay) target = (rand3 < qc.thS4) ? 1 : 0;
            else target = (rand3 < qc.thD[2][0]) ? 9 : (rand3 < qc.thD[2][1]) ? 8 : 7;
        } else {
            if (sDecay) target = 0;
            else target = (rand3 < qc.thD[3][0]) ? 8 : (rand3 < qc.thD[3][1]) ? 7 : 6;
        }
#pragma unroll
        for (int k = 0; k < NS; ++k) w[k] = {k == target ? 1. : 0., 0.};
    }
    if (qc.renorm) {                                                        // :706-712
        double popS = (w[0].re * w[0].re + w[0].im * w[0].im) + (w[1].re * w[1].re + w[1].im * w[1].im);
        double popP = 0., popD = 0.;
#pragma unroll
        for (int k = 2; k < 6; ++k) popP = popP + (w[k].re * w[k].re + w[k].im * w[k].im);
#pragma unroll
        for (int k = 6; k < 12; ++k) popD = popD + (w[k].re * w[k].re + w[k].im * w[k].im);
        const double tot = popS + popP + popD;
#pragma unroll
        for (int k = 0; k < NS; ++k) w[k] = renorm_div<F>(w[k], tot);
    }
    return kick;
}

template <bool F>
__global__ __launch_bounds__(256) void k_substeps(SubstepArgs a) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= a.n) return;
    const int S = a.S;
    double x = a.R[i], y = a.R[S + i], z = a.R[2 * S + i];
    double vx = a.V[i], vy = a.V[S + i], vz = a.V[2 * S + i];
    double fx, fy, fz;
    if (a.nseg > 1) {        // forces() left segment partials: canonical sum (slot_sum16)
        fx = slot_sum16(a.Fpart + i, (size_t)3 * S, a.nseg);
        fy = slot_sum16(a.Fpart + S + i, (size_t)3 * S, a.nseg);
        fz = slot_sum16(a.Fpart + 2 * S + i, (size_t)3 * S, a.nseg);
        a.F[i] = fx; a.F[S + i] = fy; a.F[2 * S + i] = fz;
    } else {
        fx = a.F[i]; fy = a.F[S + i]; fz = a.F[2 * S + i];
    }
    double tPart = a.tPart[i];
    cxd w[NS];
    if (a.do_qt) {
#pragma unroll
        for (int k = 0; k < NS; ++k) w[k] = {a.psi[(size_t)(2 * k) * S + i], a.psi[(size_t)(2 * k + 1) * S + i]};
    }
    const double L = a.L;
    const double dt = a.qc.dtQ;
    const double DT = 0.5 * dt;                                  // step(): step_R(0.5*dt) :426
    const uint64_t gid = a.gid0 + (uint64_t)i;
    for (int s = 0; s < a.nsub; ++s) {
        if (a.do_step) {
            const bool moving = a.t[s] > 0;                      // step_R :360
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                if (moving) {                                    // :362-367
                    x += DT * vx; y += DT * vy; z += DT * vz;
                } else {                                         // :372-378
                    x += DT * vx + DT * DT * fx;
                    y += DT * vy + DT * DT * fy;
                    z += DT * vz + DT * DT * fz;
                }
                if (x < 0) x += L;                               // :381-389
                if (x > L) x -= L;
                if (y < 0) y += L;
                if (y > L) y -= L;
                if (z < 0) z += L;
                if (z > L) z -= L;
                if (half == 0) {                                 // step_V(dt) :398-409
                    vx += dt * fx; vy += dt * fy; vz += dt * fz;
                }
            }
        }
        if (a.do_qt) {
            const double kick = qstep_ion<F>(a.qc, a.expDet[s], vx, tPart, w, gid, a.q0 + (uint64_t)s, a.U, S, i);
            vx = vx + kick;                                      // :705
        }
    }
    a.R[i] = x; a.R[S + i] = y; a.R[2 * S + i] = z;
    {
        const double lo = -0.125 * L, hi = 1.125 * L;
        if (!(x >= lo && x <= hi && y >= lo && y <= hi && z >= lo && z <= hi)) *a.oor = 1;
    }
    a.V[i] = vx; a.V[S + i] = vy; a.V[2 * S + i] = vz;
    if (a.do_qt) {
        a.tPart[i] = tPart;
#pragma unroll
        for (int k = 0; k < NS; ++k) {
            a.psi[(size_t)(2 * k) * S + i] = w[k].re;
            a.psi[(size_t)(2 * k + 1) * S + i] = w[k].im;
        }
    }
}

// ------------------------------------------------------------------------------------------
// Kernel 2b: the same substeps with one ion per 16-lane group, lane k holding state k
// (4 ions per wave64).  For small N (C2: 3573 ions = 56 waves thread-per-ion, 894 waves
// here) this fills the chip; the sparse matvec row k needs y at up to three other states,
// fetched with ds_bpermute inside the group.  Every floating-point operation is the one
// k_substeps performs, in the same order (cross-lane moves are exact), so the two kernels
// are bit-identical — tests/test_gpu_parity.py checks it.
// ------------------------------------------------------------------------------------------
template <bool F>
__global__ __launch_bounds__(256) void k_substeps_lanes(SubstepArgs a, const LaneTab* __restrict__ tab) {
    const int lane = threadIdx.x & 63;
    const int k = lane & 15;                          // state index (valid when < 12)
    const int g0 = lane & ~15;                        // first lane of this ion's group
    const int iraw = blockIdx.x * 16 + (threadIdx.x >> 4);
    const bool store = iraw < a.n;
    const int i = store ? iraw : a.n - 1;             // idle groups shadow the last ion
    const bool st = k < NS;
    const QTConst& qc = a.qc;
    const int S = a.S;
    // per-lane row structure of M and kick weights
#if !MDQT_GATHER_LDS
    const int srcA = g0 + tab->colA[k], srcB = g0 + tab->colB[k], srcC = g0 + tab->colC[k];
#endif
    const int order = tab->order[k], hasB = tab->hasB[k], hasC = tab->hasC[k];
    const int dynB = tab->dynB[k], dynC = tab->dynC[k];
    const cxd cA = {tab->cAre[k], tab->cAim[k]};
    cxd cB = {tab->cBre[k], tab->cBim[k]}, cC = {tab->cCre[k], tab->cCim[k]};
    const double dynScale = tab->dynScale[k];
    const double gA = tab->gA[k], gB = tab->gB[k], dPk = tab->dP[k], hdk = tab->hd[k];
    // ion state (replicated over the group) and this lane's amplitude
    double x = a.R[i], y = a.R[S + i], z = a.R[2 * S + i];
    double vx = a.V[i], vy = a.V[S + i], vz = a.V[2 * S + i];
    double fx, fy, fz;
    if (a.nseg > 1) {        // lanes 0..2 sum component k of the segment partials, then share
        double fk = 0.;
        if (k < 3) {
            fk = slot_sum16(a.Fpart + (size_t)k * S + i, (size_t)3 * S, a.nseg);
            if (store) a.F[(size_t)k * S + i] = fk;
        }
        fx = gat(fk, g0 + 0); fy = gat(fk, g0 + 1); fz = gat(fk, g0 + 2);
    } else {
        fx = a.F[i]; fy = a.F[S + i]; fz = a.F[2 * S + i];
    }
    double tPart = a.tPart[i];
    cxd w = {0., 0.};
    if (a.do_qt && st) w = {a.psi[(size_t)(2 * k) * S + i], a.psi[(size_t)(2 * k + 1) * S + i]};
    const double L = a.L;
    const double dt = qc.dtQ;
    const double DT = 0.5 * dt;
    const uint64_t gid = a.gid0 + (uint64_t)i;
    // Philox draws u1, u2 of all substeps of the launch up front, lane k taking substeps k and
    // k + 16 (the per-substep chain then only reads LDS; jump draws stay on demand)
    __shared__ double su[16][MAXSUB][2];
    if (a.do_qt && !a.U) {
        for (int s = k; s < a.nsub; s += 16) {
            double p, q;
            philox_pair(qc, gid, a.q0 + (uint64_t)s, 0, p, q);
            su[threadIdx.x >> 4][s][0] = p;
            su[threadIdx.x >> 4][s][1] = q;
        }
    }
    __syncthreads();
#if MDQT_GATHER_LDS
    __shared__ double2 xg[256];
    const int ldsA = (threadIdx.x & ~15) + tab->colA[k], ldsB = (threadIdx.x & ~15) + tab->colB[k],
              ldsC = (threadIdx.x & ~15) + tab->colC[k];
    auto exchange = [&](cxd v, cxd& A, cxd& B, cxd& C) {
        wave_sync();
        xg[threadIdx.x] = make_double2(v.re, v.im);
        wave_sync();
        const double2 ta = xg[ldsA], tb = xg[ldsB], tc = xg[ldsC];
        A = {ta.x, ta.y}; B = {tb.x, tb.y}; C = {tc.x, tc.y};
    };
#else
    auto exchange = [&](cxd v, cxd& A, cxd& B, cxd& C) {
        A = gatc(v, srcA); B = gatc(v, srcB); C = gatc(v, srcC);
    };
#endif
    for (int s = 0; s < a.nsub; ++s) {
        if (a.do_step) {                              // step(), as in k_substeps
            const bool moving = a.t[s] > 0;
#pragma unroll
            for (int half = 0; half < 2; ++half) {
                if (moving) {
                    x += DT * vx; y += DT * vy; z += DT * vz;
                } else {
                    x += DT * vx + DT * DT * fx;
                    y += DT * vy + DT * DT * fy;
                    z += DT * vz + DT * DT * fz;
                }
                if (x < 0) x += L;
                if (x > L) x -= L;
                if (y < 0) y += L;
                if (y > L) y -= L;
                if (z < 0) z += L;
                if (z > L) z -= L;
                if (half == 0) { vx += dt * fx; vy += dt * fy; vz += dt * fz; }
            }
        }
        if (!a.do_qt) continue;
        // ---- qstep() for this ion (SpeedUp:478-712), state k on this lane ----
        const double eD = a.expDet[s];
        const double velQuant = vx * qc.pv2q;
        tPart += qc.dtQ;
        const double Tk = decay_term<F>(w, dPk);
        const double dp = qc.h * row_sum_p(Tk);
        double u1, u2;
        if (a.U) {
            u1 = a.U[i];
            u2 = a.U[(size_t)S + i];
        } else {
            u1 = su[threadIdx.x >> 4][s][0];
            u2 = su[threadIdx.x >> 4][s][1];
        }
        cxd wA, wB, wC;
        exchange(w, wA, wB, wC);
        double kick;
        if (u1 > dp) {
            // optical kick from the pre-step density matrix (:490-503)
            const double kA = rho_im(w, wA) * gA, kB = rho_im(w, wB) * gB;
            // ((p23 g0 + p14 g2) - p25 g4) - p16 g5, evaluated at lane 0 (terms of lanes 0, 1)
            const double sum1 = dpp<BCAST(0)>(((dpp<SHL(1)>(kA) + kA) - dpp<SHL(1)>(kB)) - kB);
            // ((((((p96 g8 + p105 g11) + p114 g14) + p123 g17) - p76 g6) - p85 g9) - p94 g12) - p103 g15
            // evaluated at lane 8 (terms of lanes 6..11)
            const double sum2 = dpp<BCAST(8)>(((((((kB + dpp<SHL(1)>(kB)) + dpp<SHL(2)>(kA)) + dpp<SHL(3)>(kA)) -
                                                 dpp<SHR(2)>(kA)) - dpp<SHR(1)>(kA)) - kA) - dpp<SHL(1)>(kA));
            kick = qc.kickS * sum1 * qc.dtQ * qc.gamToE + qc.kickD * sum2 * qc.dtQ * qc.gamToE;
            // this lane's row of M = I - i h H (:506-526)
            const double vq = velQuant + eD;
            const double ER = -qc.det - velQuant - eD;
            const double EL = -qc.det + velQuant + eD;
            const double E67 = (-qc.det + qc.detDP + (1 - qc.kRat) * (velQuant + eD));
            const double E1011 = (-qc.det + qc.detDP + (qc.kRat - 1) * (velQuant + eD));
            const double E89 = (-qc.det + qc.detDP - velQuant - eD - qc.kRat * (velQuant + eD));
            const double E = (k < 2) ? 0. : (k < 4) ? ER : (k < 6) ? EL : (k < 8) ? E67 : (k < 10) ? E89 : E1011;
            const double h = qc.h;
            const cxd Md = {(k >= 2 && k < 6) ? 1. + h * hdk : 1., -(h * E)};
            const double phi = 2. * vq * (1 + qc.kRat) * tPart * qc.gamToE;
            double sn, cs;
            sincos_q<F>(phi, sn, cs);
            const double as = dynScale * sn, ac = dynScale * cs;
            if (dynB) cB = {-(h * as), h * ac};       // M85 / M94
            if (dynC) cC = {h * as, h * ac};          // M58 / M49
            cxd yv = w, acc = {0., 0.};
            cxd yA = wA, yB = wB, yC = wC;
#pragma unroll
            for (int stg = 0; stg < 4; ++stg) {
                double dpy = dp;
                if (stg > 0) {
                    const double Ty = decay_term<F>(yv, dPk);
                    dpy = qc.h * row_sum_p(Ty);
                    exchange(yv, yA, yB, yC);
                }
                const double pref = inv_sqrt_1m<F>(dpy);
                const cxd tA = cmulT<F>(cA, yA), tB = cmulT<F>(cB, yB), tC = cmulT<F>(cC, yC), tD = cmulT<F>(Md, yv);
                // ascending-column row sum (order patterns of LaneTab)
                const cxd second = (order == 3) ? tB : tD;
                const cxd third = (order == 3) ? tD : tB;
                cxd ws = cadd(tA, second);
                if (hasB) ws = cadd(ws, third);
                if (hasC) ws = cadd(ws, tC);
                const double step = (stg == 2) ? h : qc.dtHalf;
                const cxd kk = {kstage<F>(qc.invh, pref, ws.re, yv.re), kstage<F>(qc.invh, pref, ws.im, yv.im)};
                if (stg == 0) {
                    acc = kk;
                } else if (stg < 3) {
                    acc = {axpy<F>(3., kk.re, acc.re), axpy<F>(3., kk.im, acc.im)};
                } else {
                    const cxd sum = {acc.re + kk.re, acc.im + kk.im};
                    w = {axpy<F>(h, sum.re / 8, w.re), axpy<F>(h, sum.im / 8, w.im)};
                }
                if (stg < 3) yv = {axpy<F>(step, kk.re, w.re), axpy<F>(step, kk.im, w.im)};
            }
        } else {                                      // quantum jump (:573-703)
            tPart = 0;
            const double nk = w.re * w.re + w.im * w.im;
            const double n3 = dpp<BCAST(2)>(nk), n4 = dpp<BCAST(3)>(nk), n5 = dpp<BCAST(4)>(nk), n6 = dpp<BCAST(5)>(nk);
            const double tot = n3 + n4 + n5 + n6;
            const double prob3 = n3 / tot, prob4 = n4 / tot, prob5 = n5 / tot;
            const double rand2 = u2;
            double randDOrS, randDir, rand3, dummy;
            draw_pair(qc, a.U, S, i, gid, a.q0 + (uint64_t)s, 1, randDOrS, randDir);
            draw_pair(qc, a.U, S, i, gid, a.q0 + (uint64_t)s, 2, rand3, dummy);
            (void)dummy;
            const bool sDecay = !(randDOrS < qc.pD);
            if (!sDecay) kick = (randDir < 0.5) ? qc.vKickDP : -qc.vKickDP;
            else kick = (randDir < 0.5) ? qc.vKick : -qc.vKick;
            int target;
            if (rand2 < prob3) {
                if (sDecay) target = 1;
                else target = (rand3 < qc.thD[0][0]) ? 11 : (rand3 < qc.thD[0][1]) ? 10 : 9;
            } else if (rand2 < prob3 + prob4) {
                if (sDecay) target = (rand3 < qc.thS3) ? 0 : 1;
                else target = (rand3 < qc.thD[1][0]) ? 10 : (rand3 < qc.thD[1][1]) ? 9 : 8;
            } else if (rand2 < prob3 + prob4 + prob5) {
                if (sDecay) target = (rand3 < qc.thS4) ? 1 : 0;
                else target = (rand3 < qc.thD[2][0]) ? 9 : (rand3 < qc.thD[2][1]) ? 8 : 7;
            } else {
                if (sDecay) target = 0;
                else target = (rand3 < qc.thD[3][0]) ? 8 : (rand3 < qc.thD[3][1]) ? 7 : 6;
            }
            w = {k == target ? 1. : 0., 0.};
        }
        if (qc.renorm) {                              // :706-712
            // (popS + popP) + popD with popS = n0 + n1, popP = ((n2 + n3) + n4) + n5,
            // popD = ((((n6 + n7) + n8) + n9) + n10) + n11: row shifts build the three partial
            // chains at lanes 0, 2 and 6 at once, broadcasts combine them (k_substeps' order)
            const double nk = w.re * w.re + w.im * w.im;
            const double c1 = nk + dpp<SHL(1)>(nk);
            const double c3 = (c1 + dpp<SHL(2)>(nk)) + dpp<SHL(3)>(nk);
            const double c5 = (c3 + dpp<SHL(4)>(nk)) + dpp<SHL(5)>(nk);
            const double tot = (dpp<BCAST(0)>(c1) + dpp<BCAST(2)>(c3)) + dpp<BCAST(6)>(c5);
            w = renorm_div<F>(w, tot);
        }
        vx = vx + kick;
    }
    if (store) {
        if (k == 0) {
            a.R[i] = x; a.R[S + i] = y; a.R[2 * S + i] = z;
            const double lo = -0.125 * L, hi = 1.125 * L;
            if (!(x >= lo && x <= hi && y >= lo && y <= hi && z >= lo && z <= hi)) *a.oor = 1;
            a.V[i] = vx; a.V[S + i] = vy; a.V[2 * S + i] = vz;
            if (a.do_qt) a.tPart[i] = tPart;
        }
        if (a.do_qt && st) {
            a.psi[(size_t)(2 * k) * S + i] = w.re;
            a.psi[(size_t)(2 * k + 1) * S + i] = w.im;
        }
    }
}

hipError_t launch_substeps(const SubstepArgs& a, const LaneTab* tab, int mode, int fast, hipStream_t s,
                           hipEvent_t ev0, hipEvent_t ev1, int* instance) {
    if (a.n <= 0 || a.nsub <= 0) return hipSuccess;
    if (mode == 0) mode = (a.n < kLaneKernelMaxIons) ? 2 : 1;
    if (instance) *instance = (mode == 2 ? QTK_EXACT_LANES : QTK_EXACT_THREAD) + (fast ? 1 : 0);
    const dim3 gl((a.n + 15) / 16), gt((a.n + 255) / 256), b(256);
    if (fast) {
        if (mode == 2) launch_timed(k_substeps_lanes<true>, gl, b, s, ev0, ev1, a, tab);
        else launch_timed(k_substeps<true>, gt, b, s, ev0, ev1, a);
    } else {
        if (mode == 2) launch_timed(k_substeps_lanes<false>, gl, b, s, ev0, ev1, a, tab);
        else launch_timed(k_substeps<false>, gt, b, s, ev0, ev1, a);
    }
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// Observables (output(), SpeedUp:917-1032).  Deterministic fixed-shape reductions.
// ------------------------------------------------------------------------------------------
constexpr int RT = 1024;

__device__ __forceinline__ double block_sum(double v, double* sh) {
    const int t = threadIdx.x;
    sh[t] = v;
    __syncthreads();
    for (int w = RT / 2; w > 0; w >>= 1) {
        if (t < w) sh[t] = sh[t] + sh[t + w];
        __syncthreads();
    }
    const double r = sh[0];
    __syncthreads();
    return r;
}

__global__ __launch_bounds__(RT) void k_sum_vx(const double* __restrict__ V, int n, double* out, double* avg,
                                                int N) {
    __shared__ double sh[RT];
    double acc = 0.;
    for (int i = threadIdx.x; i < n; i += RT) acc += V[i];
    const double r = block_sum(acc, sh);
    if (threadIdx.x == 0) {
        out[0] = r;
        if (avg) avg[0] = N > 0 ? r / (double)N : 0.;   // velXAvg (:938) on the device (world 1)
    }
}

// output()'s per-ion columns in one array [4][n]: vx and the S / P / D populations of
// statePopulationsVsVTime (:1010-1024), the host loop's operations and order (pumping model 3:
// P = 2, 3; D = 4)
__global__ __launch_bounds__(256) void k_output_pack(const double* __restrict__ V, const double* __restrict__ psi,
                                                     int n, int S, int model, double* __restrict__ out) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    auto nrm = [&](int k) {
        const double re = psi[(size_t)(2 * k) * S + i], im = psi[(size_t)(2 * k + 1) * S + i];
        return re * re + im * im;
    };
    out[i] = V[i];
    out[(size_t)n + i] = nrm(0) + nrm(1);
    if (model == 3) {
        out[2 * (size_t)n + i] = nrm(2) + nrm(3);
        out[3 * (size_t)n + i] = nrm(4);
    } else {
        out[2 * (size_t)n + i] = nrm(2) + nrm(3) + nrm(4) + nrm(5);
        out[3 * (size_t)n + i] = nrm(6) + nrm(7) + nrm(8) + nrm(9) + nrm(10) + nrm(11);
    }
}

hipError_t launch_output_pack(const double* V, const double* psi, int n, int S, int model, double* out,
                              hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_output_pack, dim3((n + 255) / 256), dim3(256), 0, s, V, psi, n, S, model, out);
    return hipGetLastError();
}

__global__ __launch_bounds__(RT) void k_energy_sums(const double* __restrict__ V, int n, int S,
                                                    const double* __restrict__ vxAvg,
                                                    const double* __restrict__ urow, double* out) {
    __shared__ double sh[RT];
    const double avg = vxAvg[0];
    double ex = 0., ey = 0., ez = 0., u = 0.;
    for (int i = threadIdx.x; i < n; i += RT) {
        const double vx = V[i], vy = V[S + i], vz = V[2 * S + i];
        ex += 0.5 * ((vx - avg) * (vx - avg));                  // :939-944
        ey += 0.5 * (vy * vy);
        ez += 0.5 * (vz * vz);
        if (urow) u += urow[i];
    }
    const double rx = block_sum(ex, sh);
    const double ry = block_sum(ey, sh);
    const double rz = block_sum(ez, sh);
    const double ru = block_sum(u, sh);
    if (threadIdx.x == 0) { out[0] = rx; out[1] = ry; out[2] = rz; out[3] = ru; }
}

hipError_t launch_sum_vx(const double* V, int n, double* out, hipStream_t s, double* avg, int N) {
    hipLaunchKernelGGL(k_sum_vx, dim3(1), dim3(RT), 0, s, V, n, out, avg, N);
    return hipGetLastError();
}

hipError_t launch_energy_sums(const double* V, int n, int S, const double* vxAvg,
                              const double* urow, double* out, hipStream_t s) {
    hipLaunchKernelGGL(k_energy_sums, dim3(1), dim3(RT), 0, s, V, n, S, vxAvg, urow, out);
    return hipGetLastError();
}

// Gaussian KDE of the velocity distributions (:957-979): bin j of axis c sums, over the
// ions of chunk z in ascending order, exp(-V2 (b_j - v)^2) + exp(-V2 (b_j + v)^2).
constexpr int KT = 256;
__global__ __launch_bounds__(KT) void k_kde(const double* __restrict__ V, int n, int S,
                                            const double* __restrict__ vxAvg, double* Ppart,
                                            int chunk) {
    __shared__ double sv[KT];
    const int j = blockIdx.x * KT + threadIdx.x;
    const int c = blockIdx.y;
    const int z = blockIdx.z;
    const double V2 = kKdeV2;                                    // 1 / (2 * 0.002^2), :967
    const double b = (double)j * 0.0025;                         // vel[j], :340-344
    const double avg = (c == 0) ? vxAvg[0] : 0.;
    const int i0 = z * chunk, i1 = min(n, i0 + chunk);
    double acc = 0.;
    for (int it = i0; it < i1; it += KT) {
        __syncthreads();
        if (it + (int)threadIdx.x < i1) {
            const double v = V[(size_t)c * S + it + threadIdx.x];
            sv[threadIdx.x] = (c == 0) ? (v - avg) : v;
        }
        __syncthreads();
        const int m = min(KT, i1 - it);
        for (int k = 0; k < m; ++k) {
            const double v = sv[k];
            // exp(x) is exactly +0 for x < -745.14, i.e. for |b -+ v| >= 0.0773 (V2 d^2 >= 746.9):
            // an ion whose two terms are 0 on every bin of the wave adds exact zeros there and is
            // skipped (a wave spans 0.16 of the 5.0 bin range, an ion's terms 2 x 0.155): the same
            // sums, ~15x fewer exp.  NaN velocities still take the exp path.
            const bool near = !(fabs(b - v) >= kKdeSkip) || !(fabs(b + v) >= kKdeSkip);
            if (!__builtin_amdgcn_ballot_w64(near)) continue;
            acc += exp(-V2 * (b - v) * (b - v)) + exp(-V2 * (b + v) * (b + v));
        }
    }
    if (j < NBINS) Ppart[((size_t)z * 3 + c) * NBINS + j] = acc;
}

__global__ __launch_bounds__(256) void k_kde_reduce(const double* __restrict__ Ppart, int nchunk,
                                                    double* __restrict__ Pout) {
    const int j = blockIdx.x * 256 + threadIdx.x;
    if (j >= 3 * NBINS) return;
    double acc = Ppart[j];
    for (int z = 1; z < nchunk; ++z) acc += Ppart[(size_t)z * 3 * NBINS + j];
    Pout[j] = acc;
}

hipError_t launch_kde(const double* V, int n, int S, const double* vxAvg, double* Ppart,
                      int nchunk, double* Pout, hipStream_t s) {
    const int chunk = (n + nchunk - 1) / nchunk;
    dim3 grid((NBINS + KT - 1) / KT, 3, nchunk);
    hipLaunchKernelGGL(k_kde, grid, dim3(KT), 0, s, V, n, S, vxAvg, Ppart, chunk);
    hipLaunchKernelGGL(k_kde_reduce, dim3((3 * NBINS + 255) / 256), dim3(256), 0, s, Ppart, nchunk, Pout);
    return hipGetLastError();
}

// ------------------------------------------------------------------------------------------
// the optical-pumping programs' MD step (randomFrozenStartTag408Linear.cpp step() :377-394 =
// step_R(dt/2) :317-356, step_V(dt) :358-375 with forces() at the half-drifted positions,
// step_R(dt/2)), in two launches around forces(): the reference's operations, exact
// ------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_leapfrog_half(double* __restrict__ R, double* __restrict__ V,
                                                       const double* __restrict__ F, int n, int S, double L,
                                                       double DT, double DT2, int moving, double kick) {
    const int i = blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        const size_t k = (size_t)c * S + i;
        double v = V[k];
        const double f = F[k];
        if (kick != 0.) { v += kick * f; V[k] = v; }                 // V[c][i] += DT*F[c][i]   :366-370
        double r = R[k];
        r = moving ? r + DT * v : r + (DT * v + DT2 * f);            // :320-338
        if (r < 0) r += L;                                           // :346-354
        if (r > L) r -= L;
        R[k] = r;
    }
}

hipError_t launch_leapfrog_half(double* R, double* V, const double* F, int n, int S, double L, double DT, double DT2,
                                int moving, double kick, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_leapfrog_half, dim3((n + 255) / 256), dim3(256), 0, s, R, V, F, n, S, L, DT, DT2, moving, kick);
    return hipGetLastError();
}

}  // namespace mdqt
