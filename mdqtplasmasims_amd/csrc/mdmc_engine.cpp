// Host engine of the Monte-Carlo + MD analytics program: the C ABI of
// include/mdmc.h.  Owns the device-resident state (R, V, A, U, stored velocities), keeps the
// reference's std::mt19937 stream (its Metropolis part runs inside the device MC kernel, the
// state handed over both ways), drives the gfx950 kernels of mdmc_kernels.hip and the
// Newton-3 force kernel, and reproduces main()'s stages and files.  Every function cites the
// lines of MonteCarloFollowedByMDAndTempAnisotropy.cpp ("MCMD") it stands in for.
#include <errno.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>

#include <algorithm>
#include <random>
#include <string>
#include <vector>

#include "../../include/mdmc.h"
#include "mdqt_internal.hpp"

using namespace mdqt;

#define HIPCHK(expr)                                                                                        \
    do {                                                                                                    \
        hipError_t e_ = (expr);                                                                             \
        if (e_ != hipSuccess)                                                                               \
            return set_error("%s failed: %s (%s:%d)", #expr, hipGetErrorString(e_), __FILE__, __LINE__);   \
    } while (0)

// std::mt19937 ([rand.predef]) with the state in plain view: the same sequence as the
// reference's engine (so uniform_real_distribution / normal_distribution draw the same values
// from it), a discard that skips the tempering, and the device MC kernel's [624 words, position]
// layout without a text round trip.
struct Mt32 {
    using result_type = uint32_t;
    static constexpr result_type min() { return 0u; }
    static constexpr result_type max() { return 0xffffffffu; }
    uint32_t x[625];   // x[624] = position
    void seed(uint32_t s) {
        x[0] = s;
        for (uint32_t i = 1; i < 624; ++i) x[i] = 1812433253u * (x[i - 1] ^ (x[i - 1] >> 30)) + i;
        x[624] = 624;
    }
    void twist() {
        uint32_t* v = x;
        auto f = [](uint32_t a, uint32_t b, uint32_t m) {
            const uint32_t y = (a & 0x80000000u) | (b & 0x7fffffffu);
            return m ^ (y >> 1) ^ ((y & 1u) ? 0x9908b0dfu : 0u);
        };
        for (int k = 0; k < 227; ++k) v[k] = f(v[k], v[k + 1], v[k + 397]);
        for (int k = 227; k < 623; ++k) v[k] = f(v[k], v[k + 1], v[k - 227]);
        v[623] = f(v[623], v[0], v[396]);
        x[624] = 0;
    }
    result_type operator()() {
        if (x[624] >= 624) twist();
        uint32_t z = x[x[624]++];
        z ^= z >> 11;
        z ^= (z << 7) & 0x9d2c5680u;
        z ^= (z << 15) & 0xefc60000u;
        z ^= z >> 18;
        return z;
    }
    void discard(unsigned long long n) {
        while (n) {
            if (x[624] >= 624) twist();
            const unsigned long long k = std::min<unsigned long long>(n, 624 - x[624]);
            x[624] += (uint32_t)k;
            n -= k;
        }
    }
};

struct mdmc_ctx {
    mdmc_params p;
    int N = 0, S = 0, nbins = 0, T = 0, nt = 0, npairs = 0;
    double L = 0., rCut = 0.;
    double collisionFreq = 0.;
    int addLaserForce = 0;
    // the reference's RNG (MCMD:52-55, :87)
    Mt32 rng;
    std::uniform_real_distribution<double> uni{0., 1.};
    std::normal_distribution<double> vd;
    int dev = 0;
    hipStream_t st = nullptr;
    double *dR = nullptr, *dV = nullptr, *dA = nullptr, *dU = nullptr, *dD = nullptr;
    double* dRn = nullptr;          // positions of the next MDStep, pre-advanced by k_vv_step
    bool rnValid = false;           // dRn == stepPositions(dR, dV, dA): cleared by every other writer
    double *dSlots = nullptr, *dVS = nullptr, *dPart = nullptr, *dOut = nullptr;
    double *dTemp = nullptr, *dMom = nullptr;   // per-step observables of the run (4 / 20 per step)
    int capTemp = 0;
    int2* dPairs = nullptr;
    unsigned* dHist = nullptr;
    int* dTags = nullptr;
    uint32_t* dMT = nullptr;
    unsigned long long* dAcc = nullptr;
    double* hHits = nullptr;       // pinned ring of collision entries (i, vx, vy, vz), read by k_collide
    int hitCap = 0, hitOff = 0;
    std::string saveDir;
    // QT tagging variants (qt_model 1..3)
    int qt = 0;
    double dtQ = 0., gamToE = 0., pv2q = 0., decayRatio = 0.;
    int qtRatio = 0, pumpSteps = 0;
    QTConst qc;
    FastTab ftab;
    FastTab* dFTab = nullptr;      // [2]: by state, by lane (the same for the pumping models)
    double* dPsi = nullptr;        // [24][S] component-major (re0, im0, re1, ...), as include/mdqt.h's engine
    double* dTp = nullptr;         // [S] tPart
    int* dFlags = nullptr;
    double *dKdePart = nullptr, *dKde = nullptr;
    uint64_t qidx = 0;
    unsigned short x48[3] = {0x330E, 0xABCD, 0x1234};   // drand48's default state (no srand48 in QTT)
};

namespace {

int fail_free(mdmc_ctx* c, const char* what) {
    mdmc_destroy(c);
    return set_error("%s", what);
}

double sqrt_threshold(double rc) {   // smallest x with sqrt(x) >= rc: sqrt(r2) < rc iff r2 < x
    double x = rc * rc;
    while (x > 0 && sqrt(x) >= rc) x = nextafter(x, 0.);
    while (sqrt(x) < rc) x = nextafter(x, INFINITY);
    return x;
}

double mic_threshold(double L) {   // smallest d with fl(d / L) >= 0.5 (Newton-3 kernel, exact variant)
    double d = 0.5 * L;
    while (d > 0 && d / L >= 0.5) d = nextafter(d, 0.);
    while (d / L < 0.5) d = nextafter(d, INFINITY);
    return d;
}

// the rng state to / from the device MC kernel (the same [624 words, position] layout)
int rng_to_device(mdmc_ctx* c) {
    HIPCHK(hipMemcpyAsync(c->dMT, c->rng.x, sizeof c->rng.x, hipMemcpyHostToDevice, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}
int rng_from_device(mdmc_ctx* c) {
    HIPCHK(hipMemcpyAsync(c->rng.x, c->dMT, sizeof c->rng.x, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    if (c->rng.x[624] > 624) return set_error("device MC kernel returned a bad mt19937 position");
    return 0;
}

// calculateAccelerations (:387-448): the Newton-3 tile kernel (lDeb = 1/kappa); its slots are
// summed into A by k_vv_step
int accelerations(mdmc_ctx* c) {
    N3Args a;
    memset(&a, 0, sizeof a);
    a.R = c->dR; a.P = c->dSlots; a.pairs = c->dPairs;
    a.N = c->N; a.S = c->S; a.ntiles = c->nt; a.npairs = c->npairs;
    a.L = c->L; a.lDeb = 1. / c->p.kappa; a.Rcut = c->rCut; a.invlDeb = c->p.kappa;
    a.micT = mic_threshold(c->L); a.micGuard = 1.25 * c->L; a.guard = 0;
    a.rc2 = sqrt_threshold(c->rCut);
    // force_kernel 1: variant 2 (fast values, the reference's exact pair set), 0: exact
    HIPCHK(launch_forces_n3(a, c->p.force_kernel == 1 ? 2 : 0, c->st));
    return 0;
}

int mkdir_p(const char* d) {
    if (mkdir(d, 0777) != 0 && errno != EEXIST) return set_error("mkdir %s: %s", d, strerror(errno));
    return 0;
}

FILE* open_in(const mdmc_ctx* c, const char* name, const char* mode) {
    std::string f = c->saveDir + name;
    return fopen(f.c_str(), mode);
}

}  // namespace

extern "C" void mdmc_default_params(mdmc_params* p) {                 // MCMD:62-107
    memset(p, 0, sizeof *p);
    p->N = 4096; p->kappa = 0.5; p->Gamma = 3; p->n = 0.4; p->collisionFreq = 0.25;
    p->monteCarloSteps = 200000; p->maxRStep = 0.3; p->pairPairStep = 0.05; p->timeStep = 0.005;
    p->numPreRecordMDSteps = 200; p->numVelAutoCorrsSteps = 2500; p->numInstantaneousAnisotropySteps = 2500;
    p->numReestablishEquilSteps = 500; p->tempPercentDiff = 0.15; p->applyForceAlongOneAxisOnly = 0;
    p->beta = 26000; p->anisotropyEstablishmentTime = 10; p->anisotropyFromForcesRelaxSteps = 2000;
    p->seed = 12345; p->job = 1; p->device = -1; p->force_kernel = 1;
    p->qt_model = 0; p->tpumpreal = 0.0000002; p->detuning = -2.5; p->Om = 0.7;   // QTT 408 linear :85-87
    strcpy(p->saveDirectory, "data/");
}

extern "C" int mdmc_default_params_qt(mdmc_params* p, int model) {   // QTT:75-121
    if (!p) return set_error("mdmc_default_params_qt: NULL argument");
    if (model < 1 || model > 3) return set_error("mdmc_default_params_qt: model must be 1, 2 or 3");
    mdmc_default_params(p);
    p->n = 2;                                       // :82
    p->monteCarloSteps = 100000;                    // :98
    p->numVelAutoCorrsSteps = 1500;                 // :109
    p->qt_model = model;
    static const double tp[4] = {0, 0.0000002, 0.0000001, 0.00000005};   // 408Linear :85, 408Quad :114, 422 :85
    static const double det[4] = {0, -2.5, 0, -1}, om[4] = {0, 0.7, 2, 1.3};
    static const char* dir[4] = {"", "data408/", "dataSpinTagQuad/", "data422/"};
    p->tpumpreal = tp[model]; p->detuning = det[model]; p->Om = om[model];
    strcpy(p->saveDirectory, dir[model]);
    return 0;
}

extern "C" void mdmc_destroy(mdmc_ctx* c) {
    if (!c) return;
    (void)hipSetDevice(c->dev);
    if (c->st) (void)hipStreamSynchronize(c->st);
    void* ps[] = {c->dR, c->dV, c->dA, c->dRn, c->dU, c->dD, c->dSlots, c->dVS, c->dPart, c->dOut,
                  c->dTemp, c->dMom, c->dPairs, c->dHist, c->dTags, c->dMT, c->dAcc,
                  c->dFTab, c->dPsi, c->dTp, c->dFlags, c->dKdePart, c->dKde};
    for (void* q : ps)
        if (q) (void)hipFree(q);
    if (c->hHits) (void)hipHostFree(c->hHits);
    if (c->st) (void)hipStreamDestroy(c->st);
    delete c;
}

extern "C" int mdmc_create(const mdmc_params* p, mdmc_ctx** out) {
    if (!p || !out) return set_error("mdmc_create: NULL argument");
    *out = nullptr;
    if (p->N < 2) return set_error("N must be >= 2");
    if (p->numVelAutoCorrsSteps < 1 || p->numVelAutoCorrsSteps > 4096)
        return set_error("numVelAutoCorrsSteps must be in [1, 4096]");
    if (p->kappa <= 0 || p->Gamma <= 0 || p->timeStep <= 0 || p->pairPairStep <= 0)
        return set_error("kappa, Gamma, timeStep and pairPairStep must be positive");
    if (p->force_kernel != 0 && p->force_kernel != 1) return set_error("force_kernel must be 0 or 1");
    int ndev = 0;
    hipError_t e = hipGetDeviceCount(&ndev);
    if (e != hipSuccess || ndev < 1) return set_error("no HIP device available (%s)", hipGetErrorString(e));
    mdmc_ctx* c = new mdmc_ctx();
    c->p = *p;
    c->p.saveDirectory[sizeof(c->p.saveDirectory) - 1] = 0;
    if (p->device >= 0) {
        if (p->device >= ndev) { delete c; return set_error("device %d >= device count %d", p->device, ndev); }
        c->dev = p->device;
    } else {
        (void)hipGetDevice(&c->dev);
    }
    if (hipSetDevice(c->dev) != hipSuccess || hipStreamCreateWithFlags(&c->st, hipStreamNonBlocking) != hipSuccess) {
        delete c;
        return set_error("cannot create a HIP stream on device %d", p->device);
    }
    const int N = p->N;
    c->N = N;
    c->S = ((N + 63) / 64) * 64;
    c->T = p->numVelAutoCorrsSteps;
    c->L = pow(N * 4. * M_PI / 3., 1. / 3);                         // :73
    c->rCut = c->L / 2.;                                            // :74
    c->nbins = (int)((c->L / 2) / p->pairPairStep);                 // :83, :616
    c->collisionFreq = p->collisionFreq;
    c->rng.seed(p->seed);                                           // :53 (seed instead of random_device)
    (void)c->uni(c->rng);                                           // :55 auto random_double = uni(rng)
    c->vd = std::normal_distribution<double>(0, sqrt(1 / p->Gamma));   // :87
    c->nt = (N + 63) / 64;
    c->npairs = c->nt * (c->nt + 1) / 2;
    const size_t S = c->S, sz = S * sizeof(double);
    const int nblk = autocorr_blocks(N);
    bool ok = hipMalloc(&c->dR, 3 * sz) == hipSuccess && hipMalloc(&c->dV, 3 * sz) == hipSuccess &&
              hipMalloc(&c->dA, 3 * sz) == hipSuccess && hipMalloc(&c->dRn, 3 * sz) == hipSuccess &&
              hipMalloc(&c->dU, sz) == hipSuccess && hipMalloc(&c->dD, sz) == hipSuccess &&
              hipMalloc(&c->dSlots, 3 * sz * c->nt) == hipSuccess &&
              hipMalloc(&c->dVS, (size_t)3 * N * c->T * sizeof(double)) == hipSuccess &&
              hipMalloc(&c->dPart, (size_t)nblk * 4 * c->T * sizeof(double)) == hipSuccess &&
              hipMalloc(&c->dOut, (size_t)4 * c->T * sizeof(double)) == hipSuccess &&
              hipMalloc(&c->dPairs, (size_t)c->npairs * sizeof(int2)) == hipSuccess &&
              hipMalloc(&c->dHist, (size_t)(c->nbins > 0 ? c->nbins : 1) * sizeof(unsigned)) == hipSuccess &&
              hipMalloc(&c->dTags, (size_t)4 * N * sizeof(int)) == hipSuccess &&
              hipMalloc(&c->dMT, 625 * sizeof(uint32_t)) == hipSuccess &&
              hipMalloc(&c->dAcc, sizeof(unsigned long long)) == hipSuccess;
    if (!ok) return fail_free(c, "mdmc_create: device allocation failed");
    // the reference's globals start at zero (R, V, A, U; MCMD:110-123)
    ok = hipMemsetAsync(c->dR, 0, 3 * sz, c->st) == hipSuccess && hipMemsetAsync(c->dV, 0, 3 * sz, c->st) == hipSuccess &&
         hipMemsetAsync(c->dA, 0, 3 * sz, c->st) == hipSuccess && hipMemsetAsync(c->dU, 0, sz, c->st) == hipSuccess &&
         hipMemsetAsync(c->dVS, 0, (size_t)3 * N * c->T * sizeof(double), c->st) == hipSuccess &&
         hipMemsetAsync(c->dTags, 0, (size_t)4 * N * sizeof(int), c->st) == hipSuccess;
    std::vector<int2> h;
    h.reserve(c->npairs);
    for (int I = 0; I < c->nt; ++I)
        for (int J = I; J < c->nt; ++J) h.push_back(make_int2(I, J));
    ok = ok && hipMemcpyAsync(c->dPairs, h.data(), h.size() * sizeof(int2), hipMemcpyHostToDevice, c->st) == hipSuccess &&
         hipStreamSynchronize(c->st) == hipSuccess;
    if (!ok) return fail_free(c, "mdmc_create: device initialisation failed");
    c->hitCap = 4 * 65536;
    if (hipHostMalloc((void**)&c->hHits, (size_t)c->hitCap * 4 * sizeof(double), hipHostMallocDefault) != hipSuccess)
        return fail_free(c, "mdmc_create: pinned allocation failed");
    c->saveDir = c->p.saveDirectory;
    if (p->qt_model != 0) {
        // the QT tagging program's constants: 408 (QTT408Linear:115-121) / 422 (QTT422Linear:115-121)
        const int m = p->qt_model;
        if (m < 1 || m > 3) return fail_free(c, "mdmc_create: qt_model must be 0 .. 3");
        const double nn = p->n;
        c->qt = m;
        c->gamToE = m == 3 ? 174.07 * .894 / sqrt(nn) : 174.07 / sqrt(nn);
        c->qtRatio = m == 3 ? (int)round(87 * .894 / sqrt(nn)) : (int)round(87 / sqrt(nn));
        c->dtQ = p->timeStep / c->qtRatio;
        c->pv2q = m == 3 ? 1.1821 * pow(nn, 1. / 6) * .967 : 1.1821 * pow(nn, 1. / 6);
        c->decayRatio = m == 3 ? 0.0753 : 0.0617;
        const double tpump = p->tpumpreal * 813490 * sqrt(nn);
        c->pumpSteps = (int)round(tpump / p->timeStep);
        if (c->qtRatio < 1) return fail_free(c, "mdmc_create: QT substep ratio < 1");
        build_pump_program(m, p->detuning, p->Om, c->dtQ, c->gamToE, c->pv2q, c->decayRatio, p->seed, p->job, c->qc,
                           c->ftab);
        const int nch = (N + 255) / 256;
        ok = hipMalloc(&c->dFTab, 2 * sizeof(FastTab)) == hipSuccess &&
             hipMalloc(&c->dPsi, (size_t)24 * S * sizeof(double)) == hipSuccess &&
             hipMalloc(&c->dTp, (size_t)S * sizeof(double)) == hipSuccess &&
             hipMalloc(&c->dFlags, sizeof(int)) == hipSuccess &&
             hipMalloc(&c->dKdePart, (size_t)nch * 3 * TKDE_BINS * sizeof(double)) == hipSuccess &&
             hipMalloc(&c->dKde, (size_t)3 * TKDE_BINS * sizeof(double)) == hipSuccess;
        if (!ok) return fail_free(c, "mdmc_create: QT allocation failed");
        ok = hipMemcpyAsync(c->dFTab, &c->ftab, sizeof(FastTab), hipMemcpyHostToDevice, c->st) == hipSuccess &&
             hipMemcpyAsync(c->dFTab + 1, &c->ftab, sizeof(FastTab), hipMemcpyHostToDevice, c->st) == hipSuccess &&
             hipMemsetAsync(c->dPsi, 0, (size_t)24 * S * sizeof(double), c->st) == hipSuccess &&
             hipMemsetAsync(c->dTp, 0, (size_t)S * sizeof(double), c->st) == hipSuccess &&
             hipMemsetAsync(c->dFlags, 0, sizeof(int), c->st) == hipSuccess &&
             hipStreamSynchronize(c->st) == hipSuccess;
        if (!ok) return fail_free(c, "mdmc_create: QT initialisation failed");
    }
    *out = c;
    return 0;
}

extern "C" double mdmc_get_const(const mdmc_ctx* c, const char* n) {
    if (!c || !n) return NAN;
    if (!strcmp(n, "N")) return c->N;
    if (!strcmp(n, "L")) return c->L;
    if (!strcmp(n, "rCut")) return c->rCut;
    if (!strcmp(n, "nbins")) return c->nbins;
    if (!strcmp(n, "collisionFreq")) return c->collisionFreq;
    if (c->qt) {
        if (!strcmp(n, "plasmaToQuantumTimestepRatio")) return c->qtRatio;
        if (!strcmp(n, "quantumTimestep")) return c->dtQ;
        if (!strcmp(n, "gamToEinsteinFreq")) return c->gamToE;
        if (!strcmp(n, "plasVelToQuantVel")) return c->pv2q;
        if (!strcmp(n, "decayRatio")) return c->decayRatio;
        if (!strcmp(n, "pumpMDTimeSteps")) return c->pumpSteps;
    }
    return NAN;
}

// init() :173-203 (cubic lattice + Maxwell-Boltzmann velocities from the reference's rng),
// then calculatePotentialEnergyForParticles() :207-245
extern "C" int mdmc_init(mdmc_ctx* c) {
    if (!c) return set_error("NULL context");
    c->rnValid = false;
    const int N = c->N, S = c->S;
    const double L = c->L;
    std::vector<double> R((size_t)3 * S, 0.), V((size_t)3 * S, 0.);
    std::vector<double> psi(c->qt ? (size_t)24 * S : 0, 0.);
    int N0 = 0;
    for (int i = 0; i < round(pow(N, 1. / 3)); i++)
        for (int j = 0; j < round(pow(N, 1. / 3)); j++)
            for (int k = 0; k < round(pow(N, 1. / 3)); k++) {
                if (N0 >= N) return set_error("mdmc_init: N = %d is not a perfect cube (lattice init :182-201)", N);
                R[N0] = i * L / pow(N, 1 / 3.) + 0.5;               // :189-191
                R[S + N0] = j * L / pow(N, 1 / 3.) + 0.5;
                R[2 * S + N0] = k * L / pow(N, 1 / 3.) + 0.5;
                V[N0] = c->vd(c->rng);                              // :193-195
                V[S + N0] = c->vd(c->rng);
                V[2 * S + N0] = c->vd(c->rng);
                if (c->qt) {                                         // QTT:224-239: random S superposition
                    const double rand1 = erand48(c->x48), rand2 = erand48(c->x48);
                    const double rand3 = erand48(c->x48);
                    const double sign = rand3 < 0.5 ? -1 : 1;
                    const double rand4 = erand48(c->x48);
                    const double sign2 = rand4 < 0.5 ? -1 : 1;
                    psi[(size_t)0 * S + N0] = sqrt(rand1);                                    // re, state 0
                    psi[(size_t)2 * S + N0] = sign2 * sqrt(1 - rand1) * sqrt(rand2);          // re, state 1
                    psi[(size_t)3 * S + N0] = sign * sqrt(1 - rand1) * sqrt(1 - rand2);       // im, state 1
                }
                N0++;
            }
    if (N0 != N) return set_error("mdmc_init: N = %d is not a perfect cube (lattice init :182-201)", N);
    HIPCHK(hipSetDevice(c->dev));
    HIPCHK(hipMemcpyAsync(c->dR, R.data(), R.size() * sizeof(double), hipMemcpyHostToDevice, c->st));
    HIPCHK(hipMemcpyAsync(c->dV, V.data(), V.size() * sizeof(double), hipMemcpyHostToDevice, c->st));
    HIPCHK(hipMemsetAsync(c->dA, 0, (size_t)3 * S * sizeof(double), c->st));
    HIPCHK(launch_particle_potentials(c->dR, N, S, L, c->p.kappa, c->rCut, c->dU, c->st));
    if (c->qt) {
        HIPCHK(hipMemcpyAsync(c->dPsi, psi.data(), psi.size() * sizeof(double), hipMemcpyHostToDevice, c->st));
        HIPCHK(hipMemsetAsync(c->dTp, 0, (size_t)S * sizeof(double), c->st));
        c->qidx = 0;
    }
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

// MonteCarloStep() x nsteps (:315-382) on the device with the reference's mt19937 stream
extern "C" int mdmc_monte_carlo(mdmc_ctx* c, int nsteps, long long* accepted) {
    if (!c) return set_error("NULL context");
    c->rnValid = false;
    if (nsteps < 0) return set_error("nsteps < 0");
    HIPCHK(hipSetDevice(c->dev));
    if (rng_to_device(c)) return -1;
    HIPCHK(hipMemsetAsync(c->dAcc, 0, sizeof(unsigned long long), c->st));
    MCArgs a;
    a.R = c->dR; a.U = c->dU; a.D = c->dD; a.mt = c->dMT; a.accepted = c->dAcc;
    a.N = c->N; a.S = c->S;
    a.L = c->L; a.kappa = c->p.kappa; a.rCut = c->rCut; a.maxRStep = c->p.maxRStep; a.Gamma = c->p.Gamma;
    a.micT = mic_threshold(c->L);
    a.fast = c->p.force_kernel == 1;
    a.rc2 = sqrt_threshold(c->rCut);
    for (int done = 0; done < nsteps;) {                      // bounded launches
        a.nsteps = std::min(10000, nsteps - done);
        HIPCHK(launch_monte_carlo(a, c->st));
        done += a.nsteps;
    }
    unsigned long long acc = 0;
    HIPCHK(hipMemcpyAsync(&acc, c->dAcc, sizeof acc, hipMemcpyDeviceToHost, c->st));
    if (rng_from_device(c)) return -1;
    if (accepted) *accepted = (long long)acc;
    return 0;
}

// One MDStep() (:504-511) queued on the stream: stepPositions, calculateAccelerations,
// stepVelocities.  The collision rolls and Maxwellian draws of the step are state-independent,
// so the host makes them (the reference's rng, its order :474-482) while the device runs.
static int md_step_async(mdmc_ctx* c) {
    const int N = c->N;
    const double dt = c->p.timeStep;
    if (!c->rnValid)                                                                          // :452-467
        HIPCHK(launch_vv_positions(c->dR, c->dV, c->dA, c->dRn, N, c->S, dt, c->L, c->st));
    std::swap(c->dR, c->dRn);
    if (accelerations(c)) return -1;                                                          // :508
    int nh = 0;
    double* hits = nullptr;
    if (dt * c->collisionFreq <= 0) {
        // every roll misses (uni >= 0): each is one generate_canonical, i.e. two mt19937 words
        c->rng.discard(2ull * N);
    } else {
        if (c->hitOff + N > c->hitCap) {           // ring wrap: the queued readers must be done
            HIPCHK(hipStreamSynchronize(c->st));
            c->hitOff = 0;
        }
        hits = c->hHits + (size_t)4 * c->hitOff;
        for (int i = 0; i < N; i++) {
            const double collRoll = c->uni(c->rng);
            if (collRoll < dt * c->collisionFreq) {
                double* e = hits + 4 * (size_t)nh++;
                e[0] = i;
                e[1] = c->vd(c->rng);
                e[2] = c->vd(c->rng);
                e[3] = c->vd(c->rng);
            }
        }
        c->hitOff += nh;
    }
    VVArgs v;
    v.V = c->dV; v.A = c->dA; v.slots = c->dSlots; v.nslots = c->nt; v.R = c->dR; v.Rn = c->dRn; v.L = c->L;
    v.hits = hits; v.nhits = nh; v.N = N; v.S = c->S;
    v.laser = c->addLaserForce; v.oneAxis = c->p.applyForceAlongOneAxisOnly;
    v.dt = dt; v.p6 = pow(10, -6); v.beta = c->p.beta; v.sqrtn = sqrt(c->p.n);
    HIPCHK(launch_vv_velocities(v, c->st));                                                   // :469-502
    c->rnValid = true;
    return 0;
}

extern "C" int mdmc_md_steps(mdmc_ctx* c, int nsteps) {
    if (!c) return set_error("NULL context");
    HIPCHK(hipSetDevice(c->dev));
    for (int k = 0; k < nsteps; ++k)
        if (md_step_async(c)) return -1;
    HIPCHK(hipStreamSynchronize(c->st));
    c->hitOff = 0;
    return 0;
}

extern "C" int mdmc_set_collision_freq(mdmc_ctx* c, double f) {
    if (!c) return set_error("NULL context");
    c->collisionFreq = f;
    return 0;
}
extern "C" int mdmc_set_laser_force(mdmc_ctx* c, int on) {
    if (!c) return set_error("NULL context");
    c->addLaserForce = on ? 1 : 0;
    return 0;
}

// recordPairPairCorr (:584-635): the histogram on the device, the normalisation here
static int pair_corr_host(mdmc_ctx* c, std::vector<double>& g) {
    HIPCHK(hipSetDevice(c->dev));
    const int nb = c->nbins;
    g.assign(nb > 0 ? nb : 0, 0.);
    if (nb <= 0) return 0;
    std::vector<unsigned> h(nb);
    HIPCHK(hipMemsetAsync(c->dHist, 0, nb * sizeof(unsigned), c->st));
    HIPCHK(launch_pair_hist(c->dR, c->N, c->S, c->L, c->p.pairPairStep, nb, c->dHist, c->st));
    HIPCHK(hipMemcpyAsync(h.data(), c->dHist, nb * sizeof(unsigned), hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    const int N = c->N;
    const double ps = c->p.pairPairStep;
    for (int i = 0; i < nb; i++) {                               // :627-635
        if (i == 0) g[i] = (double)h[i] / (N * 4 / 3 * M_PI * ps * ps * ps);
        else g[i] = (double)h[i] / (N * 3 * ps * ps * ps * i * i);
    }
    return 0;
}

extern "C" int mdmc_pair_corr(mdmc_ctx* c, double* g, int cap, int* nbins) {
    if (!c) return set_error("NULL context");
    std::vector<double> v;
    if (pair_corr_host(c, v)) return -1;
    if (nbins) *nbins = (int)v.size();
    if (g) {
        if (cap < (int)v.size()) return set_error("mdmc_pair_corr: buffer holds %d < %d bins", cap, (int)v.size());
        memcpy(g, v.data(), v.size() * sizeof(double));
    }
    return 0;
}

extern "C" int mdmc_record_velocities(mdmc_ctx* c, int k) {      // :513-523
    if (!c) return set_error("NULL context");
    if (k < 0 || k >= c->T) return set_error("mdmc_record_velocities: step %d outside [0, %d)", k, c->T);
    HIPCHK(hipSetDevice(c->dev));
    HIPCHK(launch_store_velocities(c->dV, c->N, c->S, c->T, k, c->dVS, c->st));
    return 0;
}

extern "C" int mdmc_set_velocity_store(mdmc_ctx* c, const double* vs) {
    if (!c || !vs) return set_error("mdmc_set_velocity_store: NULL argument");
    HIPCHK(hipSetDevice(c->dev));
    HIPCHK(hipMemcpyAsync(c->dVS, vs, (size_t)3 * c->N * c->T * sizeof(double), hipMemcpyHostToDevice, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

// recordVAF, recordLongViscAutoCorr, recordVCubeAutoCorr, recordVFourthAutoCorr (:655-807)
extern "C" int mdmc_autocorrelations(mdmc_ctx* c, double* out) {
    if (!c || !out) return set_error("mdmc_autocorrelations: NULL argument");
    HIPCHK(hipSetDevice(c->dev));
    const double G = c->p.Gamma;
    const double c2 = 3 / (G * G), c4 = 3 * 9 / (G * G * G * G);   // :710, :785
    HIPCHK(launch_autocorr(c->dVS, c->N, c->T, c2, c4, c->dPart, c->dOut, c->st));
    HIPCHK(hipMemcpyAsync(out, c->dOut, (size_t)4 * c->T * sizeof(double), hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

static void temps_from_sums(const mdmc_ctx* c, const double* s, double* out4) {
    out4[0] = s[0] / (c->N * 3);                                 // recordTemperature :535-543
    out4[1] = s[1] / c->N;                                       // recordTempForEachAxis :567-576
    out4[2] = s[2] / c->N;
    out4[3] = s[3] / c->N;
}

extern "C" int mdmc_temperatures(mdmc_ctx* c, double out4[4]) {
    if (!c || !out4) return set_error("mdmc_temperatures: NULL argument");
    HIPCHK(hipSetDevice(c->dev));
    double s[4];
    HIPCHK(launch_temperatures(c->dV, c->N, c->S, c->dOut, c->st));
    HIPCHK(hipMemcpyAsync(s, c->dOut, sizeof s, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    temps_from_sums(c, s, out4);
    return 0;
}

extern "C" int mdmc_anisotropize(mdmc_ctx* c) {                  // :548-558
    if (!c) return set_error("NULL context");
    c->rnValid = false;
    HIPCHK(hipSetDevice(c->dev));
    HIPCHK(launch_anisotropize(c->dV, c->N, c->S, c->p.tempPercentDiff, c->st));
    return 0;
}

// tagParticles (:810-921): needs vx only, consumes the reference's rng on the host
extern "C" int mdmc_tag_particles(mdmc_ctx* c, int* tags4) {
    if (!c) return set_error("NULL context");
    HIPCHK(hipSetDevice(c->dev));
    const int N = c->N;
    std::vector<double> vx(N);
    std::vector<int> t((size_t)4 * N);
    HIPCHK(hipMemcpyAsync(vx.data(), c->dV, N * sizeof(double), hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    const double Gamma = c->p.Gamma;
    const double vT = sqrt(1 / Gamma);                           // :814
    double roll;
    for (int i = 0; i < N; i++) {
        const double currVx = vx[i];
        int one, two, three, four;
        if (currVx < -3 * vT) one = 0;                           // :819-838
        else if (currVx > 3 * vT) one = 1;
        else { roll = c->uni(c->rng); one = roll < (.5 + currVx / vT / 6); }
        const double c2 = .5 / 9 / vT / vT;                      // :840-864
        roll = c->uni(c->rng);
        if (currVx < -3 * vT || currVx > 3 * vT) two = !(roll < .5);
        else two = roll < (c2 * currVx * currVx);
        const double c3 = .5 / 27 / vT / vT / vT;                // :868-888
        if (currVx < -3 * vT) three = 0;
        else if (currVx > 3 * vT) three = 1;
        else { roll = c->uni(c->rng); three = roll < (.5 + c3 * currVx * currVx * currVx); }
        const double c4 = .5 / 81 / vT / vT / vT / vT;           // :892-916
        roll = c->uni(c->rng);
        if (currVx < -3 * vT || currVx > 3 * vT) four = !(roll < .5);
        else four = roll < (c4 * currVx * currVx * currVx * currVx);
        t[i] = one; t[(size_t)N + i] = two; t[(size_t)2 * N + i] = three; t[(size_t)3 * N + i] = four;
    }
    HIPCHK(hipMemcpyAsync(c->dTags, t.data(), t.size() * sizeof(int), hipMemcpyHostToDevice, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    if (tags4) memcpy(tags4, t.data(), t.size() * sizeof(int));
    return 0;
}

static void moments_from_sums(const mdmc_ctx* c, const double* m, double* out16) {   // :972-998
    const double G = c->p.Gamma;
    for (int t = 0; t < 4; ++t) {
        const unsigned num = (unsigned)m[5 * t + 4];
        out16[4 * t] = m[5 * t] / num;
        out16[4 * t + 1] = m[5 * t + 1] / num;
        out16[4 * t + 1] -= 1 / (G);
        out16[4 * t + 2] = m[5 * t + 2] / num;
        out16[4 * t + 3] = m[5 * t + 3] / num;
        out16[4 * t + 3] -= 3 / (G * G);
    }
}

extern "C" int mdmc_tagged_moments(mdmc_ctx* c, double out16[16]) {
    if (!c || !out16) return set_error("mdmc_tagged_moments: NULL argument");
    HIPCHK(hipSetDevice(c->dev));
    double m[20];
    HIPCHK(launch_tag_moments(c->dV, c->dTags, c->N, c->dOut, c->st));
    HIPCHK(hipMemcpyAsync(m, c->dOut, sizeof m, hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    moments_from_sums(c, m, out16);
    return 0;
}

extern "C" int mdmc_get_state(mdmc_ctx* c, double* R, double* V, double* A, double* U) {
    if (!c) return set_error("NULL context");
    HIPCHK(hipSetDevice(c->dev));
    const int N = c->N, S = c->S;
    double* src[3] = {c->dR, c->dV, c->dA};
    double* dst[3] = {R, V, A};
    for (int q = 0; q < 3; ++q) {
        if (!dst[q]) continue;
        for (int k = 0; k < 3; ++k)
            HIPCHK(hipMemcpyAsync(dst[q] + (size_t)k * N, src[q] + (size_t)k * S, N * sizeof(double),
                                  hipMemcpyDeviceToHost, c->st));
    }
    if (U) HIPCHK(hipMemcpyAsync(U, c->dU, N * sizeof(double), hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

extern "C" int mdmc_set_state(mdmc_ctx* c, const double* R, const double* V, const double* A, const double* U) {
    if (!c) return set_error("NULL context");
    c->rnValid = false;
    HIPCHK(hipSetDevice(c->dev));
    const int N = c->N, S = c->S;
    if (R)   // the kernels' division-free minimum image needs |dx| < 1.25 L: the box of :262-271, :459-464
        for (size_t k = 0; k < (size_t)3 * N; ++k)
            if (!(R[k] >= 0 && R[k] <= c->L)) return set_error("mdmc_set_state: position %zu = %g outside [0, L]", k, R[k]);
    double* dst[3] = {c->dR, c->dV, c->dA};
    const double* src[3] = {R, V, A};
    for (int q = 0; q < 3; ++q) {
        if (!src[q]) continue;
        for (int k = 0; k < 3; ++k)
            HIPCHK(hipMemcpyAsync(dst[q] + (size_t)k * S, src[q] + (size_t)k * N, N * sizeof(double),
                                  hipMemcpyHostToDevice, c->st));
    }
    if (U) HIPCHK(hipMemcpyAsync(c->dU, U, N * sizeof(double), hipMemcpyHostToDevice, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

// ---- QT tagging variants ----
static int need_qt(const mdmc_ctx* c, const char* what) {
    if (!c) return set_error("NULL context");
    if (!c->qt) return set_error("%s: the context has no QT (qt_model 0)", what);
    return 0;
}

// qstep() x n (QTT:555-756): the pumping model's fused QT substeps on this system's velocities
// (no drift: the MD steps move the ions), in launches of up to MAXSUB substeps
static int qsteps_async(mdmc_ctx* c, int n) {
    while (n > 0) {
        const int m = n < MAXSUB ? n : MAXSUB;
        SubstepArgs a;
        memset(&a, 0, sizeof a);
        a.R = c->dR; a.V = c->dV; a.F = c->dA; a.Fpart = nullptr; a.nseg = 1;
        a.psi = c->dPsi; a.tPart = c->dTp; a.oor = c->dFlags;
        a.n = c->N; a.S = c->S; a.gid0 = 0; a.q0 = c->qidx;
        a.nsub = m; a.do_step = 0; a.do_qt = 1; a.U = nullptr;
        a.L = c->L;
        a.qc = c->qc;
        HIPCHK(launch_substeps_r(a, c->dFTab, 0, c->st));
        c->qidx += (uint64_t)m;
        n -= m;
    }
    return 0;
}

extern "C" int mdmc_qsteps(mdmc_ctx* c, int n) {
    if (need_qt(c, "mdmc_qsteps")) return -1;
    HIPCHK(hipSetDevice(c->dev));
    if (qsteps_async(c, n)) return -1;
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

// tagParticles (QTT:1022-1067 / 422:992-1034): the spin-up measurement of include/mdqt.h's
// k_tag_spin_up (Philox draws 6, 7 of the current qstep index); the tags drive the moments
extern "C" int mdmc_tag_qt(mdmc_ctx* c, int* tags, int* n_up) {
    if (need_qt(c, "mdmc_tag_qt")) return -1;
    HIPCHK(hipSetDevice(c->dev));
    const int N = c->N;
    HIPCHK(launch_tag_spin_up(c->dPsi, N, c->S, 0, c->qidx, c->qc, c->dTags, c->st));
    std::vector<int> h((size_t)N);
    HIPCHK(hipMemcpyAsync(h.data(), c->dTags, (size_t)N * sizeof(int), hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    int cnt = 0;
    for (int i = 0; i < N; ++i) cnt += h[i];
    if (tags) memcpy(tags, h.data(), (size_t)N * sizeof(int));
    if (n_up) *n_up = cnt;
    return 0;
}

// recordTaggedParticleMoments (QTT:1069-1138): moments from the device sums of tag set 0,
// distributions from k_tagged_kde (queued; dist == NULL skips them)
static int tagged_moments_qt_queue(mdmc_ctx* c, double* sums_dev, bool dist) {
    HIPCHK(launch_tag_moments(c->dV, c->dTags, c->N, sums_dev, c->st));
    if (dist) HIPCHK(launch_tagged_kde(c->dV, c->dTags, c->N, c->S, c->dKdePart, c->dKde, c->st));
    return 0;
}
static void moments_qt_from_sums(const double* m, double* out4) {   // :1106-1109
    const unsigned num = (unsigned)m[4];
    out4[0] = m[0] / num; out4[1] = m[1] / num; out4[2] = m[2] / num; out4[3] = m[3] / num;
}

extern "C" int mdmc_tagged_moments_qt(mdmc_ctx* c, double out4[4], double* dist) {
    if (need_qt(c, "mdmc_tagged_moments_qt")) return -1;
    if (!out4) return set_error("mdmc_tagged_moments_qt: NULL argument");
    HIPCHK(hipSetDevice(c->dev));
    if (tagged_moments_qt_queue(c, c->dOut, dist != nullptr)) return -1;
    double m[20];
    HIPCHK(hipMemcpyAsync(m, c->dOut, sizeof m, hipMemcpyDeviceToHost, c->st));
    if (dist) HIPCHK(hipMemcpyAsync(dist, c->dKde, (size_t)3 * TKDE_BINS * sizeof(double), hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    moments_qt_from_sums(m, out4);
    return 0;
}

extern "C" int mdmc_get_psi(mdmc_ctx* c, double* psi) {             // [N][12][2]
    if (need_qt(c, "mdmc_get_psi")) return -1;
    if (!psi) return set_error("mdmc_get_psi: NULL argument");
    HIPCHK(hipSetDevice(c->dev));
    const int N = c->N, S = c->S;
    std::vector<double> h((size_t)24 * S);
    HIPCHK(hipMemcpyAsync(h.data(), c->dPsi, h.size() * sizeof(double), hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    for (int i = 0; i < N; ++i)
        for (int k = 0; k < 24; ++k) psi[(size_t)24 * i + k] = h[(size_t)k * S + i];
    return 0;
}

extern "C" int mdmc_set_psi(mdmc_ctx* c, const double* psi) {
    if (need_qt(c, "mdmc_set_psi")) return -1;
    if (!psi) return set_error("mdmc_set_psi: NULL argument");
    HIPCHK(hipSetDevice(c->dev));
    const int N = c->N, S = c->S;
    std::vector<double> h((size_t)24 * S, 0.);
    for (int i = 0; i < N; ++i)
        for (int k = 0; k < 24; ++k) h[(size_t)k * S + i] = psi[(size_t)24 * i + k];
    HIPCHK(hipMemcpyAsync(c->dPsi, h.data(), h.size() * sizeof(double), hipMemcpyHostToDevice, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    return 0;
}

extern "C" int mdmc_setup_directories(mdmc_ctx* c) {            // main() :1037-1058
    if (!c) return set_error("NULL context");
    std::string d = c->p.saveDirectory;
    if (mkdir_p(d.c_str())) return -1;
    char nb[256];
    if (c->qt)                                                     // QTT:1153
        snprintf(nb, sizeof nb, "Gamma%dKappa%dNumIons%dPumpTime%dDet%dOm%dDensity%d", (unsigned)(c->p.Gamma * 100),
                 (unsigned)(c->p.kappa * 100), (unsigned)(c->N), (unsigned)(1000000000. * c->p.tpumpreal),
                 (unsigned)(100. * fabs(c->p.detuning)), (unsigned)(100. * c->p.Om), (unsigned)(10. * c->p.n));
    else
        snprintf(nb, sizeof nb, "Gamma%dKappa%dNumIons%d", (unsigned)(c->p.Gamma * 100), (unsigned)(c->p.kappa * 100),
                 (unsigned)(c->N));
    d += nb;
    if (mkdir_p(d.c_str())) return -1;
    snprintf(nb, sizeof nb, "/job%d/", c->p.job);
    d += nb;
    if (mkdir_p(d.c_str())) return -1;
    c->saveDir = d;
    return 0;
}

extern "C" const char* mdmc_save_directory(const mdmc_ctx* c) { return c ? c->saveDir.c_str() : ""; }

static int write_pair_corr(mdmc_ctx* c, int stepNum) {          // :639-651
    std::vector<double> g;
    if (pair_corr_host(c, g)) return -1;
    char name[256];
    snprintf(name, sizeof name, "pairPairCorrStepNum%d.dat", stepNum);
    FILE* fa = open_in(c, name, "w");
    if (!fa) return set_error("cannot open %s%s", c->saveDir.c_str(), name);
    for (int i = 0; i < (int)g.size(); i++) fprintf(fa, "%lg\t%lg\n", i * c->p.pairPairStep, g[i]);
    fclose(fa);
    return 0;
}

// per-step observables buffered on the device, written when a stage ends
static int ensure_step_buffers(mdmc_ctx* c, int steps) {
    if (steps <= c->capTemp) return 0;
    if (c->dTemp) HIPCHK(hipFree(c->dTemp));
    if (c->dMom) HIPCHK(hipFree(c->dMom));
    c->dTemp = nullptr; c->dMom = nullptr;
    HIPCHK(hipMalloc(&c->dTemp, (size_t)steps * 4 * sizeof(double)));
    HIPCHK(hipMalloc(&c->dMom, (size_t)steps * 20 * sizeof(double)));
    c->capTemp = steps;
    return 0;
}

static int write_temp_axes(mdmc_ctx* c, const char* name, int nsteps) {   // recordTempForEachAxis :560-581
    std::vector<double> s((size_t)nsteps * 4);
    HIPCHK(hipMemcpyAsync(s.data(), c->dTemp, s.size() * sizeof(double), hipMemcpyDeviceToHost, c->st));
    HIPCHK(hipStreamSynchronize(c->st));
    FILE* fa = open_in(c, name, "a");
    if (!fa) return set_error("cannot open %s%s", c->saveDir.c_str(), name);
    for (int k = 0; k < nsteps; ++k) {
        double t4[4];
        temps_from_sums(c, &s[(size_t)4 * k], t4);
        fprintf(fa, "%lg\t%lg\t%lg\t%lg\n", k * c->p.timeStep, t4[1], t4[2], t4[3]);
    }
    fclose(fa);
    return 0;
}

static int write_autocorrelations(mdmc_ctx* c) {                // :682-691 and the three siblings
    std::vector<double> out((size_t)4 * c->T);
    if (mdmc_autocorrelations(c, out.data())) return -1;
    const char* names[4] = {"VAF.dat", "longViscAutoCorr.dat", "vCubeAutoCorr.dat", "vFourthAutoCorr.dat"};
    for (int f = 0; f < 4; ++f) {
        FILE* fa = open_in(c, names[f], "w");
        if (!fa) return set_error("cannot open %s%s", c->saveDir.c_str(), names[f]);
        for (int td = 0; td < c->T; ++td) fprintf(fa, "%lg\t%lg\n", td * c->p.timeStep, out[(size_t)f * c->T + td]);
        fclose(fa);
    }
    return 0;
}

// main() of the QT tagging programs (QTT:1140-1254)
static int run_qtt(mdmc_ctx* c, int verbose) {
    const mdmc_params& p = c->p;
    if (mdmc_setup_directories(c)) return -1;                    // :1143-1167
    if (mdmc_init(c)) return -1;                                 // steps 1-2 :1192-1196
    for (int k = 0; k < p.monteCarloSteps;) {                    // step 3 :1198-1209
        if (k % 10000 == 0) {
            if (write_pair_corr(c, k)) return -1;
            if (verbose) printf("%d\n", k);
        }
        const int next = std::min(p.monteCarloSteps, (k / 10000 + 1) * 10000);
        if (mdmc_monte_carlo(c, next - k, nullptr)) return -1;
        k = next;
    }
    for (int k = 0; k < p.numPreRecordMDSteps; k++) {            // step 4 :1211-1220
        if (verbose && k % 100 == 0) printf("%d\n", k);
        if (md_step_async(c)) return -1;
    }
    c->collisionFreq = 0;                                        // step 5 :1222-1233
    if (verbose) printf("pumpMDTimeSteps=%d\nquantumStepsPerMD=%d\n", c->pumpSteps, c->qtRatio);
    for (int k = 0; k < c->pumpSteps; k++) {
        if (qsteps_async(c, c->qtRatio)) return -1;
        if (md_step_async(c)) return -1;
    }
    if (mdmc_tag_qt(c, nullptr, nullptr)) return -1;
    const int T = c->T;                                          // step 6 :1235-1245
    std::vector<double> m(20), dist((size_t)3 * TKDE_BINS);
    FILE* fm = open_in(c, "taggedMoments.dat", "a");
    FILE* ft = open_in(c, "temperature.dat", "a");
    if (!fm || !ft) return set_error("cannot open taggedMoments.dat / temperature.dat in %s", c->saveDir.c_str());
    for (int k = 0; k < T; k++) {
        if (tagged_moments_qt_queue(c, c->dOut, true)) return -1;
        HIPCHK(hipMemcpyAsync(m.data(), c->dOut, 20 * sizeof(double), hipMemcpyDeviceToHost, c->st));
        HIPCHK(hipMemcpyAsync(dist.data(), c->dKde, dist.size() * sizeof(double), hipMemcpyDeviceToHost, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
        double mom[4];
        moments_qt_from_sums(m.data(), mom);
        fprintf(fm, "%lg\t%lg\t%lg\t%lg\t%lg\n", k * p.timeStep, mom[0], mom[1], mom[2], mom[3]);   // :1114
        char name[64];
        snprintf(name, sizeof name, "vel_distX_timestep%06d.dat", k);                                     // :1128-1136
        FILE* fd = open_in(c, name, "w");
        if (!fd) return set_error("cannot open %s%s", c->saveDir.c_str(), name);
        for (int j = 0; j < TKDE_BINS; j++) fprintf(fd, "%lg\t%lg\n", (double)(j - 2000) * 0.0025, dist[j]);
        fclose(fd);
        if (k % 100 == 0) {
            if (verbose) printf("%d\n", k);
            if (write_pair_corr(c, k)) return -1;
        }
        double t4[4];
        HIPCHK(launch_temperatures(c->dV, c->N, c->S, c->dOut, c->st));   // recordTemperature :771-792
        HIPCHK(hipMemcpyAsync(t4, c->dOut, sizeof t4, hipMemcpyDeviceToHost, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
        double tt[4];
        temps_from_sums(c, t4, tt);
        fprintf(ft, "%lg\n", tt[0]);
        if (md_step_async(c)) return -1;
        if (mdmc_record_velocities(c, k)) return -1;
    }
    fclose(fm);
    fclose(ft);
    if (write_autocorrelations(c)) return -1;                    // step 7 :1247-1251
    if (verbose) fflush(stdout);
    return 0;
}

// main() :1030-1167
extern "C" int mdmc_run(mdmc_ctx* c, int verbose) {
    if (!c) return set_error("NULL context");
    if (c->qt) return run_qtt(c, verbose);
    const mdmc_params& p = c->p;
    if (mdmc_setup_directories(c)) return -1;                    // :1037-1058
    if (mdmc_init(c)) return -1;                                 // step 1-2 :1062-1065
    for (int k = 0; k < p.monteCarloSteps;) {                    // step 3 :1068-1078
        if (k % 10000 == 0) {
            if (write_pair_corr(c, k)) return -1;
            if (verbose) printf("%d\n", k);
        }
        const int next = std::min(p.monteCarloSteps, (k / 10000 + 1) * 10000);
        if (mdmc_monte_carlo(c, next - k, nullptr)) return -1;
        k = next;
    }
    for (int k = 0; k < p.numPreRecordMDSteps; k++) {            // step 4 :1081-1089
        if (verbose && k % 100 == 0) printf("%d\n", k);
        if (md_step_async(c)) return -1;
    }
    c->collisionFreq = 0;                                        // step 5 :1093-1104
    if (mdmc_tag_particles(c, nullptr)) return -1;
    const int T = c->T;
    if (ensure_step_buffers(c, std::max(T, std::max(p.numInstantaneousAnisotropySteps,
                                                    std::max(p.anisotropyFromForcesRelaxSteps, 1 << 16))))) return -1;
    for (int k = 0; k < T; k++) {
        HIPCHK(launch_tag_moments(c->dV, c->dTags, c->N, c->dMom + (size_t)20 * k, c->st));
        if (k % 100 == 0) {
            if (verbose) printf("%d\n", k);
            if (write_pair_corr(c, k)) return -1;
        }
        HIPCHK(launch_temperatures(c->dV, c->N, c->S, c->dTemp + (size_t)4 * k, c->st));
        if (md_step_async(c)) return -1;
        if (mdmc_record_velocities(c, k)) return -1;
    }
    {   // recordTemperature (:533-545) and recordTaggedParticleMoments (:1005-1027), appended per step
        std::vector<double> s((size_t)T * 4), m((size_t)T * 20);
        HIPCHK(hipMemcpyAsync(s.data(), c->dTemp, s.size() * sizeof(double), hipMemcpyDeviceToHost, c->st));
        HIPCHK(hipMemcpyAsync(m.data(), c->dMom, m.size() * sizeof(double), hipMemcpyDeviceToHost, c->st));
        HIPCHK(hipStreamSynchronize(c->st));
        FILE* ft = open_in(c, "temperature.dat", "a");
        const char* names[4] = {"taggedVOneMoments.dat", "taggedVTwoMoments.dat", "taggedVThreeMoments.dat",
                                "taggedVFourMoments.dat"};
        FILE* fm[4];
        for (int t = 0; t < 4; ++t) fm[t] = open_in(c, names[t], "a");
        if (!ft || !fm[0] || !fm[1] || !fm[2] || !fm[3]) return set_error("cannot open the stage-5 files");
        for (int k = 0; k < T; ++k) {
            double t4[4], m16[16];
            temps_from_sums(c, &s[(size_t)4 * k], t4);
            moments_from_sums(c, &m[(size_t)20 * k], m16);
            for (int t = 0; t < 4; ++t)
                fprintf(fm[t], "%lg\t%lg\t%lg\t%lg\t%lg\n", k * p.timeStep, m16[4 * t], m16[4 * t + 1], m16[4 * t + 2],
                        m16[4 * t + 3]);
            fprintf(ft, "%lg\n", t4[0]);
        }
        fclose(ft);
        for (int t = 0; t < 4; ++t) fclose(fm[t]);
    }
    if (write_autocorrelations(c)) return -1;                    // step 6 :1107-1110
    if (mdmc_anisotropize(c)) return -1;                         // step 7 :1115-1123
    for (int k = 0; k < p.numInstantaneousAnisotropySteps; k++) {
        HIPCHK(launch_temperatures(c->dV, c->N, c->S, c->dTemp + (size_t)4 * k, c->st));
        if (md_step_async(c)) return -1;
    }
    if (write_temp_axes(c, "TemperaturesAlongAxesInstantaneous.dat", p.numInstantaneousAnisotropySteps)) return -1;
    c->collisionFreq = 0.25;                                     // :1125-1135
    for (int k = 0; k < p.numReestablishEquilSteps; k++) {
        if (verbose && k % 100 == 0) printf("%d\n", k);
        if (md_step_async(c)) return -1;
    }
    c->addLaserForce = 1;                                        // step 8 :1138-1151
    c->collisionFreq = 0;
    const int nest = (int)round(.8 * p.anisotropyEstablishmentTime * sqrt(p.n) / p.timeStep);   // :106
    if (ensure_step_buffers(c, std::max(nest, c->capTemp))) return -1;
    for (int k = 0; k < nest; k++) {
        HIPCHK(launch_temperatures(c->dV, c->N, c->S, c->dTemp + (size_t)4 * k, c->st));
        if (md_step_async(c)) return -1;
    }
    if (write_temp_axes(c, "TemperaturesAlongAxesDuringForcePeriod.dat", nest)) return -1;
    c->addLaserForce = 0;                                        // :1155-1165
    for (int k = 0; k < p.anisotropyFromForcesRelaxSteps; k++) {
        HIPCHK(launch_temperatures(c->dV, c->N, c->S, c->dTemp + (size_t)4 * k, c->st));
        if (md_step_async(c)) return -1;
    }
    if (write_temp_axes(c, "TemperaturesAlongAxesAfterForcePeriod.dat", p.anisotropyFromForcesRelaxSteps)) return -1;
    if (verbose) fflush(stdout);
    return 0;
}
