/*
 * ORACLE — TEST INFRASTRUCTURE ONLY (see mdqt_oracle.h for the rules and the pinning status).
 *
 * Plain-C restatement of laserCoolingPlusExpansionMDQTSpeedUp.cpp ("SpeedUp").  Each function
 * cites the SpeedUp lines it follows.  The floating-point operation order of the reference is
 * kept wherever the C++ source fixes it; where Armadillo 7.600.1 chooses the order internally
 * (dense complex products), the natural ascending-index order is used and the result is
 * "parity unpinned" at the ulp level.
 *
 * Build: oracle/Makefile (gcc -O2 -ffp-contract=off -fopenmp).  No FMA contraction, no
 * fast-math: the x86-64 reference build (g++ -O3, no -march) has neither.
 */
#define _GNU_SOURCE
#include "mdqt_oracle.h"

#include <errno.h>
#include <math.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <sys/stat.h>
#ifdef _OPENMP
#include <omp.h>
#endif

#define NS 12           /* numStates, SpeedUp:153 */
#define TIMESTEP 0.002  /* SpeedUp:80 */
#define NBINS 2001      /* SpeedUp:120-123 */
#define NINTERVALV 13   /* numberOfIntervalV, SpeedUp:105 */

typedef struct { double re, im; } cx;

static inline cx cx_make(double re, double im) { cx z; z.re = re; z.im = im; return z; }
/* std::complex<double> operator* without fast-math: (ac - bd, ad + bc) */
static inline cx cx_mul(cx a, cx b) { return cx_make(a.re * b.re - a.im * b.im, a.re * b.im + a.im * b.re); }
static inline cx cx_add(cx a, cx b) { return cx_make(a.re + b.re, a.im + b.im); }
static inline cx cx_sub(cx a, cx b) { return cx_make(a.re - b.re, a.im - b.im); }
static inline cx cx_conj(cx a) { return cx_make(a.re, -a.im); }
static inline cx cx_rscale(double s, cx a) { return cx_make(s * a.re, s * a.im); }
static inline double cx_norm(cx a) { return a.re * a.re + a.im * a.im; } /* libstdc++ std::norm */

struct orc_sim {
    orc_params p;
    /* derived constants */
    double gamToE, dtQ, plasVelToQuantVel, r, kRat, vKick, vKickDP, lDeb, L;
    int ratio;
    double gs[18];
    int cs_a[18], cs_b[18];           /* cs[k] = |a><b| (0-based), SpeedUp:1163-1180 */
    cx decay[NS][NS];                 /* decayMatrix, SpeedUp:1203 */
    cx hamDecay[NS][NS];              /* hamDecayTerm, SpeedUp:1202 */
    cx hamCoupNoT[NS][NS];            /* hamCouplingTermNoTimeDep, SpeedUp:1206-1215 */
    /* state (SpeedUp:126-152) */
    int N, cap;
    double *R, *V, *F;                /* [3][cap] */
    double *psi;                      /* [cap][12][2] */
    double *tPart;                    /* [cap] */
    double *Vholder;                  /* [13][3][cap] (VZERO files; zero for new runs) */
    double t;
    int c0;
    unsigned counter;
    double Epot, Epot0;
    double vel[NBINS];
    uint64_t x48;                     /* drand48 state */
    uint64_t qidx;                    /* number of qstep() calls (Philox counter) */
    char saveDirectory[1024];
    uint64_t* ion_ids;                /* Philox ion key of local ion i (NULL: i); sampled-ion checks */
    int n_ion_ids;
    int* spinUp;                      /* SpinUpList (randomFrozenStartTag408Linear.cpp:105), orc_run_pump */
    int nSpinUp;
    double* vaHold;                   /* Vholder of Zfunc (:938-961) */
};

/* ------------------------------------------------------------------------------------------ */
/* RNG                                                                                          */
/* ------------------------------------------------------------------------------------------ */

/* glibc srand48: X = (seed << 16) | 0x330E (upper 32 bits of the long ignored) */
uint64_t orc_srand48_state(uint32_t seed) { return (((uint64_t)seed) << 16) | 0x330Eull; }

/* glibc drand48: X <- (0x5DEECE66D X + 0xB) mod 2^48, returns X / 2^48 exactly */
double orc_drand48_next(uint64_t* x) {
    *x = (0x5DEECE66Dull * (*x) + 0xBull) & 0xFFFFFFFFFFFFull;
    return ldexp((double)(*x), -48);
}

/* Philox4x32-10 (Salmon et al., SC'11; Random123 constants) */
void orc_philox4x32_10(const uint32_t ctr[4], const uint32_t key[2], uint32_t out[4]) {
    uint32_t c0 = ctr[0], c1 = ctr[1], c2 = ctr[2], c3 = ctr[3];
    uint32_t k0 = key[0], k1 = key[1];
    for (int r = 0; r < 10; ++r) {
        uint64_t p0 = (uint64_t)0xD2511F53u * c0;
        uint64_t p1 = (uint64_t)0xCD9E8D57u * c2;
        uint32_t hi0 = (uint32_t)(p0 >> 32), lo0 = (uint32_t)p0;
        uint32_t hi1 = (uint32_t)(p1 >> 32), lo1 = (uint32_t)p1;
        uint32_t n0 = hi1 ^ c1 ^ k0, n1 = lo1, n2 = hi0 ^ c3 ^ k1, n3 = lo0;
        c0 = n0; c1 = n1; c2 = n2; c3 = n3;
        if (r < 9) { k0 += 0x9E3779B9u; k1 += 0xBB67AE85u; }
    }
    out[0] = c0; out[1] = c1; out[2] = c2; out[3] = c3;
}

/* The build's counter-based stream: key = (seed, job), counter = (ion, qstep_lo, qstep_hi,
 * draw/2); a uniform in [0,1) with 53 random bits from two 32-bit words. draw = 0..4 ↔ u1..u5. */
double orc_philox_uniform(uint32_t seed, uint32_t job, uint64_t ion, uint64_t qstep, int draw) {
    uint32_t ctr[4] = {(uint32_t)ion, (uint32_t)qstep, (uint32_t)(qstep >> 32),
                       ((uint32_t)(ion >> 32) << 8) | (uint32_t)(draw >> 1)};
    uint32_t key[2] = {seed, job};
    uint32_t o[4];
    orc_philox4x32_10(ctr, key, o);
    uint32_t hi = (draw & 1) ? o[2] : o[0];
    uint32_t lo = (draw & 1) ? o[3] : o[1];
    uint64_t b = ((((uint64_t)hi) << 32) | lo) >> 11;
    return (double)b * 0x1.0p-53;
}

typedef struct {
    int mode;            /* 0 drand48, 1 philox, 2 tape */
    uint64_t* x48;
    uint32_t seed, job;
    uint64_t ion, qidx;
    const double* tape;
    int n;               /* draws consumed */
} rngsrc;

static double draw(rngsrc* g) {
    double u;
    if (g->mode == 0) u = orc_drand48_next(g->x48);
    else if (g->mode == 1) u = orc_philox_uniform(g->seed, g->job, g->ion, g->qidx, g->n);
    else u = g->tape[g->n];
    g->n++;
    return u;
}

/* ------------------------------------------------------------------------------------------ */
/* construction: derived constants and the constant QT operators                                */
/* ------------------------------------------------------------------------------------------ */

void orc_default_params(orc_params* p) {
    memset(p, 0, sizeof(*p));
    p->Ge = 0.1; p->tmax = 30; p->density = 2; p->sig0 = 4.0; p->Te = 19.0; p->fracOfSig = 0;
    p->detuning = -1; p->detuningDP = 1; p->Om = 1; p->OmDP = 1;
    p->N0 = 3500; p->newRun = 1; p->c0 = 0; p->sampleFreq = 40; p->reNormalizewvFns = 0;
    p->qt_enabled = 1; p->rng_mode = 0; p->seed = 12345; p->job = 1; p->nthreads = 1;
    strcpy(p->saveDirectory, "dataLaserCool/");
    p->tpumpreal = 0.0000002; p->tstartV0 = 15;          /* randomFrozenStartTag408Linear.cpp:58, :78 */
}

static int reserve(orc_sim* s, int cap) {
    if (cap <= s->cap) return 0;
    int oldcap = s->cap;
    double* R = calloc((size_t)3 * cap, sizeof(double));
    double* V = calloc((size_t)3 * cap, sizeof(double));
    double* F = calloc((size_t)3 * cap, sizeof(double));
    double* psi = calloc((size_t)24 * cap, sizeof(double));
    double* tp = calloc((size_t)cap, sizeof(double));
    double* vh = calloc((size_t)NINTERVALV * 3 * cap, sizeof(double));
    if (!R || !V || !F || !psi || !tp || !vh) return -1;
    for (int k = 0; k < 3; ++k) {
        if (oldcap) {
            memcpy(R + (size_t)k * cap, s->R + (size_t)k * oldcap, sizeof(double) * oldcap);
            memcpy(V + (size_t)k * cap, s->V + (size_t)k * oldcap, sizeof(double) * oldcap);
            memcpy(F + (size_t)k * cap, s->F + (size_t)k * oldcap, sizeof(double) * oldcap);
        }
    }
    if (oldcap) {
        memcpy(psi, s->psi, sizeof(double) * 24 * (size_t)oldcap);
        memcpy(tp, s->tPart, sizeof(double) * (size_t)oldcap);
        for (int c = 0; c < NINTERVALV * 3; ++c)
            memcpy(vh + (size_t)c * cap, s->Vholder + (size_t)c * oldcap, sizeof(double) * oldcap);
    }
    free(s->R); free(s->V); free(s->F); free(s->psi); free(s->tPart); free(s->Vholder);
    s->R = R; s->V = V; s->F = F; s->psi = psi; s->tPart = tp; s->Vholder = vh; s->cap = cap;
    return 0;
}

orc_sim* orc_create(const orc_params* p) {
    orc_sim* s = calloc(1, sizeof(orc_sim));
    if (!s) return NULL;
    s->p = *p;
    /* SpeedUp:79-85, :146; the pumping programs: randomFrozenStartTag408Linear.cpp:67-75, :118
       (408Quad :69-77, :121) round the ratio; randomFrozenStartTag422Linear.cpp:66-74, :116 scale
       gamma by .894 and the velocity conversion by .967, D/S decay ratio 0.0754 */
    const int m = p->qt_model;
    s->gamToE = m == 3 ? 174.07 * .894 / sqrt(p->density) : 174.07 / sqrt(p->density);
    s->ratio = m == 0 ? (int)ceil(34.81 / sqrt(p->density))
             : m == 3 ? (int)round(34.81 * .894 / sqrt(p->density)) : (int)round(34.81 / sqrt(p->density));
    s->dtQ = TIMESTEP / s->ratio;
    s->plasVelToQuantVel = m == 3 ? 1.1821 * pow(p->density, 1. / 6) * .967 : 1.1821 * pow(p->density, 1. / 6);
    /* SpeedUp:146-149 */
    s->r = m == 3 ? 0.0754 : 0.0617;
    s->kRat = 0.395;
    s->vKick = 0.001208 / s->plasVelToQuantVel;
    s->vKickDP = s->vKick * s->kRat;
    /* SpeedUp:295-297 (also readConditions :787-788) */
    s->lDeb = 1. / sqrt(3. * p->Ge);
    s->L = pow(p->N0 * 4. * M_PI / 3., 0.333333333);
    /* SpeedUp:1163-1180: cs[k] = wvFn_a * wvFn_b.t()  (1-based names -> 0-based) */
    static const int A[18] = {1, 1, 0, 0, 1, 0, 6, 7, 8, 7, 8, 9, 8, 9, 10, 9, 10, 11};
    static const int B[18] = {2, 3, 3, 4, 4, 5, 5, 5, 5, 4, 4, 4, 3, 3, 3, 2, 2, 2};
    for (int k = 0; k < 18; ++k) { s->cs_a[k] = A[k]; s->cs_b[k] = B[k]; }
    /* SpeedUp:1181-1198 */
    double r = s->r;
    s->gs[0] = sqrt(1.);
    s->gs[1] = sqrt(2. / 3);
    s->gs[2] = sqrt(1. / 3);
    s->gs[3] = sqrt(2. / 3);
    s->gs[4] = sqrt(1. / 3);
    s->gs[5] = sqrt(1.);
    s->gs[6] = sqrt(r * 2. / 3);
    s->gs[7] = sqrt(r * 4. / 15);
    s->gs[8] = sqrt(r * 1. / 15);
    s->gs[9] = sqrt(r * 2. / 5);
    s->gs[10] = sqrt(r * 2. / 5);
    s->gs[11] = sqrt(r * 1. / 5);
    s->gs[12] = sqrt(r * 1. / 5);
    s->gs[13] = sqrt(r * 2. / 5);
    s->gs[14] = sqrt(r * 2. / 5);
    s->gs[15] = sqrt(r * 1. / 15);
    s->gs[16] = sqrt(r * 4. / 15);
    s->gs[17] = sqrt(r * 2. / 3);
    /* SpeedUp:1201-1204: cs[j].t()*cs[j] = |b><b| */
    memset(s->decay, 0, sizeof(s->decay));
    memset(s->hamDecay, 0, sizeof(s->hamDecay));
    for (int j = 0; j < 18; ++j) {
        int b = s->cs_b[j];
        double g2 = s->gs[j] * s->gs[j];
        /* hamDecayTerm - 1./2*I*(g^2 |b><b|):  (0,0.5)*(g2,0) = (0, 0.5*g2) */
        s->hamDecay[b][b] = cx_sub(s->hamDecay[b][b], cx_make(0., 0.5 * g2));
        s->decay[b][b] = cx_add(s->decay[b][b], cx_make(g2, 0.));
    }
    /* SpeedUp:1206-1215: -1.*cs[k].t()*gs[k]*Om/2 (SP), .../2/sqrt(r) (DP); cs.t() = |b><a| */
    memset(s->hamCoupNoT, 0, sizeof(s->hamCoupNoT));
    for (int k = 0; k < 6; ++k) {
        if (k != 1 && k != 3) {
            double v = ((-1. * s->gs[k]) * p->Om) / 2;
            s->hamCoupNoT[s->cs_b[k]][s->cs_a[k]] = cx_add(s->hamCoupNoT[s->cs_b[k]][s->cs_a[k]], cx_make(v, 0.));
        }
    }
    for (int k = 6; k < 18; ++k) {
        if (k != 8 && k != 11 && k != 7 && k != 10 && k != 13 && k != 16) {
            double v = (((-1. * s->gs[k]) * p->OmDP) / 2) / sqrt(r);
            s->hamCoupNoT[s->cs_b[k]][s->cs_a[k]] = cx_add(s->hamCoupNoT[s->cs_b[k]][s->cs_a[k]], cx_make(v, 0.));
        }
    }
    for (int i = 0; i < NBINS; ++i) s->vel[i] = (double)i * 0.0025; /* SpeedUp:340-344 */
    s->x48 = orc_srand48_state(p->seed);                             /* SpeedUp:1219 */
    s->t = 0.;
    s->c0 = p->c0;
    s->counter = 0;
    s->Epot = s->Epot0 = 0.;
    s->qidx = 0;
    strncpy(s->saveDirectory, p->saveDirectory, sizeof(s->saveDirectory) - 1);
    int cap0 = p->N0 + 1000 + 8 * (int)sqrt((double)p->N0) + 64;
    if (reserve(s, cap0)) { orc_destroy(s); return NULL; }
    return s;
}

void orc_destroy(orc_sim* s) {
    if (!s) return;
    free(s->R); free(s->V); free(s->F); free(s->psi); free(s->tPart); free(s->Vholder);
    free(s->ion_ids);
    free(s->spinUp);
    free(s->vaHold);
    free(s);
}

double orc_get_const(const orc_sim* s, const char* n) {
    if (!strcmp(n, "gamToEinsteinFreq")) return s->gamToE;
    if (!strcmp(n, "quantumTimestep")) return s->dtQ;
    if (!strcmp(n, "plasmaToQuantumTimestepRatio")) return s->ratio;
    if (!strcmp(n, "plasVelToQuantVel")) return s->plasVelToQuantVel;
    if (!strcmp(n, "vKick")) return s->vKick;
    if (!strcmp(n, "vKickDP")) return s->vKickDP;
    if (!strcmp(n, "lDeb")) return s->lDeb;
    if (!strcmp(n, "L")) return s->L;
    if (!strcmp(n, "decayRatioD5Halves")) return s->r;
    if (!strcmp(n, "kRat")) return s->kRat;
    if (!strncmp(n, "gs", 2)) return s->gs[atoi(n + 2)];
    if (!strncmp(n, "decay", 5)) return s->decay[atoi(n + 5)][atoi(n + 5)].re;
    return NAN;
}

/* ------------------------------------------------------------------------------------------ */
/* init (SpeedUp:289-348)                                                                        */
/* ------------------------------------------------------------------------------------------ */

int orc_init(orc_sim* s) {
    double L = s->L;
    double N9L = (unsigned)(9. * 9. * 9. * (L * L * L) * 3. / (4. * M_PI)); /* :299 */
    s->N = 0;
    for (long i = 0; i < N9L; i++) {                                          /* :303 */
        double x = 9. * L * orc_drand48_next(&s->x48) - 4. * L;
        double y = 9. * L * orc_drand48_next(&s->x48) - 4. * L;
        double z = 9. * L * orc_drand48_next(&s->x48) - 4. * L;
        if (x <= L && y <= L && z <= L && x > 0 && y > 0 && z > 0) {         /* :308 */
            if (s->N >= s->cap && reserve(s, s->cap + s->cap / 4 + 1024)) return -1;
            int n = s->N, c = s->cap;
            s->R[n] = x; s->R[c + n] = y; s->R[2 * c + n] = z;
            s->V[n] = 0.; s->V[c + n] = 0.; s->V[2 * c + n] = 0.;
            double rand1 = orc_drand48_next(&s->x48);                        /* :317-328 */
            double rand2 = orc_drand48_next(&s->x48);
            double rand3 = orc_drand48_next(&s->x48);
            double sign = 1;
            if (rand3 < 0.5) sign = -1;
            double rand4 = orc_drand48_next(&s->x48);
            double sign2 = 1;
            if (rand4 < 0.5) sign2 = -1;
            double* ps = s->psi + (size_t)24 * n;                             /* :329-332 */
            memset(ps, 0, 24 * sizeof(double));
            ps[0] = sqrt(rand1);
            ps[2] = sign2 * sqrt(1 - rand1) * sqrt(rand2);
            ps[3] = sign * sqrt(1 - rand1) * sqrt(1 - rand2);
            s->tPart[n] = 0;
            s->N++;
        }
    }
    s->Epot = orc_epotential(s);                                              /* :345-347 */
    s->Epot0 = s->Epot;
    s->c0 = -1;
    s->t = 0.;
    s->qidx = 0;
    return 0;
}

/* ------------------------------------------------------------------------------------------ */
/* state access                                                                                 */
/* ------------------------------------------------------------------------------------------ */

int orc_get_N(const orc_sim* s) { return s->N; }
double orc_get_time(const orc_sim* s) { return s->t; }
void orc_set_time(orc_sim* s, double t) { s->t = t; }
/* the QT constants of another program driving the same qstep (the MC + MD tagging programs,
   MonteCarloFollowedByQTTagging408Linear.cpp:115-121, 422Linear.cpp:115-121) */
void orc_set_qt_constants(orc_sim* s, double dtQ, double gamToE, double pv2q, double r) {
    s->dtQ = dtQ; s->gamToE = gamToE; s->plasVelToQuantVel = pv2q; s->r = r;
}
uint64_t orc_get_qstep_index(const orc_sim* s) { return s->qidx; }
void orc_set_qstep_index(orc_sim* s, uint64_t q) { s->qidx = q; }
void orc_set_drand48_state(orc_sim* s, uint64_t x) { s->x48 = x & 0xFFFFFFFFFFFFull; }
uint64_t orc_get_drand48_state(const orc_sim* s) { return s->x48; }
int orc_get_counters(const orc_sim* s, int* c0, unsigned* counter, double* Epot, double* Epot0) {
    if (c0) *c0 = s->c0;
    if (counter) *counter = s->counter;
    if (Epot) *Epot = s->Epot;
    if (Epot0) *Epot0 = s->Epot0;
    return 0;
}
const char* orc_save_directory(const orc_sim* s) { return s->saveDirectory; }

void orc_set_state(orc_sim* s, int N, const double* R, const double* V, size_t ld,
                   const double* psi, const double* tPart, double t) {
    if (N > s->cap) reserve(s, N + 64);
    s->N = N;
    int c = s->cap;
    for (int k = 0; k < 3; ++k)
        for (int i = 0; i < N; ++i) {
            if (R) s->R[(size_t)k * c + i] = R[(size_t)k * ld + i];
            if (V) s->V[(size_t)k * c + i] = V[(size_t)k * ld + i];
        }
    if (psi) memcpy(s->psi, psi, sizeof(double) * 24 * (size_t)N);
    if (tPart) memcpy(s->tPart, tPart, sizeof(double) * (size_t)N);
    s->t = t;
}

void orc_set_forces(orc_sim* s, const double* F, size_t ld) {
    for (int k = 0; k < 3; ++k)
        for (int i = 0; i < s->N; ++i) s->F[(size_t)k * s->cap + i] = F[(size_t)k * ld + i];
}

void orc_get_state(const orc_sim* s, double* R, double* V, double* F, size_t ld,
                   double* psi, double* tPart, double* t) {
    int c = s->cap, N = s->N;
    for (int k = 0; k < 3; ++k)
        for (int i = 0; i < N; ++i) {
            if (R) R[(size_t)k * ld + i] = s->R[(size_t)k * c + i];
            if (V) V[(size_t)k * ld + i] = s->V[(size_t)k * c + i];
            if (F) F[(size_t)k * ld + i] = s->F[(size_t)k * c + i];
        }
    if (psi) memcpy(psi, s->psi, sizeof(double) * 24 * (size_t)N);
    if (tPart) memcpy(tPart, s->tPart, sizeof(double) * (size_t)N);
    if (t) *t = s->t;
}

/* ------------------------------------------------------------------------------------------ */
/* forces (SpeedUp:192-236) and Epotential (SpeedUp:244-281)                                     */
/* ------------------------------------------------------------------------------------------ */

/* One pair, i's view: the body of SpeedUp:213-230.  In the single-thread reference the
 * Newton-3 scatter F[j] -= f(i,j) equals F[j] += f(j,i) exactly (minimum image, dr and
 * ftotal are sign-symmetric in IEEE arithmetic), so F_i is the ascending-j left-to-right sum
 * of f(i,j) — which is what the owner-computes loop below evaluates. */
void orc_forces_rows(int N, int lo, int hi, double L, double lDeb, const double* R, size_t ld,
                     double* F, int nthreads) {
    const double Rcut = L / 2.;
    const double* X = R; const double* Y = R + ld; const double* Z = R + 2 * ld;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 16) num_threads(nthreads > 0 ? nthreads : 1)
#endif
    for (int i = lo; i < hi; i++) {
        double Fx = 0., Fy = 0., Fz = 0.;
        double rx = X[i], ry = Y[i], rz = Z[i];
        for (int j = 0; j < N; j++) {
            if (j == i) continue;
            double dx = rx - X[j];
            double dy = ry - Y[j];
            double dz = rz - Z[j];
            dx -= L * round(dx / L);
            dy -= L * round(dy / L);
            dz -= L * round(dz / L);
            double dr = sqrt(dx * dx + dy * dy + dz * dz);
            if (dr > 0 && dr < Rcut) {
                double ftotal = (1. / dr + 1. / lDeb) * exp(-dr / lDeb) / (dr * dr);
                Fx += dx * ftotal;
                Fy += dy * ftotal;
                Fz += dz * ftotal;
            }
        }
        F[i] = Fx; F[ld + i] = Fy; F[2 * ld + i] = Fz;
    }
    (void)nthreads;
}

/* rows idx[0..nidx) of the same pair terms (every j), F is [3][nidx], summed with Neumaier
 * compensation: at N ~ 1e6 a plain ascending sum carries ~N eps of rounding of its own, so the
 * large-N GPU checks compare sampled ions against these nearly exact rows. */
void orc_forces_index(int N, double L, double lDeb, const double* R, size_t ld, const int* idx, int nidx,
                      double* F, int nthreads) {
    const double Rcut = L / 2.;
    const double* X = R; const double* Y = R + ld; const double* Z = R + 2 * ld;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
#endif
    for (int k = 0; k < nidx; k++) {
        const int i = idx[k];
        double S[3] = {0., 0., 0.}, C[3] = {0., 0., 0.};   /* Neumaier sum and its compensation */
        double rx = X[i], ry = Y[i], rz = Z[i];
        for (int j = 0; j < N; j++) {                                            /* SpeedUp:211-230 */
            if (j == i) continue;
            double dx = rx - X[j];
            double dy = ry - Y[j];
            double dz = rz - Z[j];
            dx -= L * round(dx / L);
            dy -= L * round(dy / L);
            dz -= L * round(dz / L);
            double dr = sqrt(dx * dx + dy * dy + dz * dz);
            if (dr > 0 && dr < Rcut) {
                double ftotal = (1. / dr + 1. / lDeb) * exp(-dr / lDeb) / (dr * dr);
                const double t[3] = {dx * ftotal, dy * ftotal, dz * ftotal};
                for (int c = 0; c < 3; ++c) {
                    const double u = S[c] + t[c];
                    C[c] += (fabs(S[c]) >= fabs(t[c])) ? (S[c] - u) + t[c] : (t[c] - u) + S[c];
                    S[c] = u;
                }
            }
        }
        F[k] = S[0] + C[0]; F[nidx + k] = S[1] + C[1]; F[2 * (size_t)nidx + k] = S[2] + C[2];
    }
    (void)nthreads;
}

/* rows idx[0..nidx) of the pair potential exp(-r/lDeb)/r over all j inside L/2 (SpeedUp:256-266, the terms
 * Epotential() sums), compensated (Neumaier) sum: U[k] = U_idx[k] (sampled-ion checks at large N) */
void orc_potentials_index(int N, double L, double lDeb, const double* R, size_t ld, const int* idx, int nidx,
                          double* U, int nthreads) {
    const double Rcut = L / 2.;
    const double* X = R; const double* Y = R + ld; const double* Z = R + 2 * ld;
#ifdef _OPENMP
#pragma omp parallel for schedule(dynamic, 1) num_threads(nthreads > 0 ? nthreads : 1)
#endif
    for (int k = 0; k < nidx; k++) {
        const int i = idx[k];
        double S = 0., C = 0.;
        double rx = X[i], ry = Y[i], rz = Z[i];
        for (int j = 0; j < N; j++) {
            if (j == i) continue;
            double dx = rx - X[j];
            double dy = ry - Y[j];
            double dz = rz - Z[j];
            dx -= L * round(dx / L);
            dy -= L * round(dy / L);
            dz -= L * round(dz / L);
            double dr = sqrt(dx * dx + dy * dy + dz * dz);
            if (dr > 0 && dr < Rcut) {
                const double t = exp(-dr / lDeb) / (dr);                                  /* :265 */
                const double u = S + t;
                C += (fabs(S) >= fabs(t)) ? (S - u) + t : (t - u) + S;
                S = u;
            }
        }
        U[k] = S + C;
    }
    (void)nthreads;
}

void orc_set_ion_ids(orc_sim* s, const uint64_t* ids, int n) {
    free(s->ion_ids);
    s->ion_ids = NULL;
    s->n_ion_ids = 0;
    if (!ids || n <= 0) return;
    s->ion_ids = (uint64_t*)malloc(sizeof(uint64_t) * (size_t)n);
    memcpy(s->ion_ids, ids, sizeof(uint64_t) * (size_t)n);
    s->n_ion_ids = n;
}

void orc_forces_raw(int N, double L, double lDeb, const double* R, size_t ld, double* F, int nthreads) {
    orc_forces_rows(N, 0, N, L, lDeb, R, ld, F, nthreads);
}

void orc_forces(orc_sim* s) {
    orc_forces_raw(s->N, s->L, s->lDeb, s->R, (size_t)s->cap, s->F, s->p.nthreads);
}

double orc_epotential_raw(int N, double L, double lDeb, const double* R, size_t ld) {
    const double Rcut = L / 2.;
    const double* X = R; const double* Y = R + ld; const double* Z = R + 2 * ld;
    double Epot = 0.;
    for (int i = 0; i < N; i++) {
        double rx = X[i], ry = Y[i], rz = Z[i];
        for (int j = i + 1; j < N; j++) {
            double dx = rx - X[j];
            double dy = ry - Y[j];
            double dz = rz - Z[j];
            dx -= L * round(dx / L);
            dy -= L * round(dy / L);
            dz -= L * round(dz / L);
            double dr = sqrt(dx * dx + dy * dy + dz * dz);
            if (dr > 0 && dr < Rcut) Epot += exp(-dr / lDeb) / (dr);
        }
    }
    Epot /= (double)N;
    return Epot;
}

double orc_epotential(orc_sim* s) {
    s->Epot = orc_epotential_raw(s->N, s->L, s->lDeb, s->R, (size_t)s->cap);
    return s->Epot;
}

/* ------------------------------------------------------------------------------------------ */
/* step (SpeedUp:356-430)                                                                        */
/* ------------------------------------------------------------------------------------------ */

static void step_R(orc_sim* s, double DT) {
    int c = s->cap, N = s->N;
    double L = s->L;
    double *X = s->R, *Y = s->R + c, *Z = s->R + 2 * c;
    const double *Vx = s->V, *Vy = s->V + c, *Vz = s->V + 2 * c;
    const double *Fx = s->F, *Fy = s->F + c, *Fz = s->F + 2 * c;
    if (s->t > 0) {                                               /* :360-368 */
        for (int i = 0; i < N; i++) {
            X[i] += DT * Vx[i];
            Y[i] += DT * Vy[i];
            Z[i] += DT * Vz[i];
        }
    } else {                                                      /* :370-379 */
        for (int i = 0; i < N; i++) {
            X[i] += DT * Vx[i] + DT * DT * Fx[i];
            Y[i] += DT * Vy[i] + DT * DT * Fy[i];
            Z[i] += DT * Vz[i] + DT * DT * Fz[i];
        }
    }
    for (int i = 0; i < N; i++) {                                 /* :381-389 */
        if (X[i] < 0) X[i] += L;
        if (X[i] > L) X[i] -= L;
        if (Y[i] < 0) Y[i] += L;
        if (Y[i] > L) Y[i] -= L;
        if (Z[i] < 0) Z[i] += L;
        if (Z[i] > L) Z[i] -= L;
    }
}

static void step_V(orc_sim* s, double DT) {                       /* :398-409 */
    int c = s->cap, N = s->N;
    for (int k = 0; k < 3; ++k)
        for (int i = 0; i < N; i++) s->V[(size_t)k * c + i] += DT * s->F[(size_t)k * c + i];
}

void orc_step(orc_sim* s) {                                       /* :418-430 */
    double dt = s->dtQ;
    step_R(s, 0.5 * dt);
    step_V(s, dt);
    step_R(s, 0.5 * dt);
}

/* ------------------------------------------------------------------------------------------ */
/* qstep (SpeedUp:438-717): dense literal restatement of the Armadillo algebra                  */
/* ------------------------------------------------------------------------------------------ */

static double expDetuning_of(const orc_sim* s, double t) {       /* :447 */
    const orc_params* p = &s->p;
    return 0.0126 * p->fracOfSig * p->Te * t /
           (sqrt(p->density) * p->sig0 * sqrt(1 + 0.00014314 * t * t * p->Te / (p->density * p->sig0 * p->sig0)));
}

/* Re(c * y^H * D * y), c = dtQuant*gamToEinsteinFreq (SpeedUp:484-485, :530-531) */
static double dp_of(const orc_sim* s, const cx* y, double c) {
    cx row[NS];
    for (int m = 0; m < NS; ++m) {
        cx acc = cx_make(0., 0.);
        for (int k = 0; k < NS; ++k) acc = cx_add(acc, cx_mul(cx_conj(y[k]), s->decay[k][m]));
        row[m] = acc;
    }
    cx v = cx_make(0., 0.);
    for (int m = 0; m < NS; ++m) v = cx_add(v, cx_mul(row[m], y[m]));
    return c * v.re;
}

static void matvec(cx M[NS][NS], const cx* y, cx* out) {
    for (int k = 0; k < NS; ++k) {
        cx acc = cx_make(0., 0.);
        for (int m = 0; m < NS; ++m) acc = cx_add(acc, cx_mul(M[k][m], y[m]));
        out[k] = acc;
    }
}

static int qstep_ion(const orc_sim* s, double t, double expDetuning, double* psi, double* vx,
                     double* tPart, rngsrc* g) {
    const orc_params* p = &s->p;
    const double dtQuant = s->dtQ, gamToE = s->gamToE, r = s->r, kRat = s->kRat;
    const double* gs = s->gs;
    cx wvFn[NS];
    for (int k = 0; k < NS; ++k) wvFn[k] = cx_make(psi[2 * k], psi[2 * k + 1]);   /* :480 */
    double velPlas = *vx;                                                       /* :481 */
    double velQuant = velPlas * s->plasVelToQuantVel;                           /* :482 */
    *tPart += dtQuant;                                                          /* :483 */
    double dp = dp_of(s, wvFn, dtQuant * gamToE);                               /* :484-485 */
    double rand = draw(g);                                                      /* :486 */
    double kick;
    int jumped = 0;
    (void)t;
    if (rand > dp) {                                                            /* :487 */
        /* densMatrix = wvFn*wvFn.t(); p_ab = rho(a-1,b-1) (:490-502) */
#define RHO_IM(a, b) (cx_mul(wvFn[a], cx_conj(wvFn[b])).im)
        double p23 = RHO_IM(1, 2), p14 = RHO_IM(0, 3), p25 = RHO_IM(1, 4), p16 = RHO_IM(0, 5);
        double p96 = RHO_IM(8, 5), p105 = RHO_IM(9, 4), p114 = RHO_IM(10, 3), p123 = RHO_IM(11, 2);
        double p76 = RHO_IM(6, 5), p85 = RHO_IM(7, 4), p94 = RHO_IM(8, 3), p103 = RHO_IM(9, 2);
#undef RHO_IM
        kick = 1 * s->vKick * p->Om * (p23 * gs[0] + p14 * gs[2] - p25 * gs[4] - p16 * gs[5]) * dtQuant * gamToE +
               s->vKickDP * (p->OmDP / r) *
                   (p96 * gs[8] + p105 * gs[11] + p114 * gs[14] + p123 * gs[17] - p76 * gs[6] - p85 * gs[9] -
                    p94 * gs[12] - p103 * gs[15]) * dtQuant * gamToE;              /* :503 */
        /* Hamiltonian (:506-521) */
        double totalDetRightSP = -p->detuning - velQuant - expDetuning;
        double totalDetLeftSP = -p->detuning + velQuant + expDetuning;
        double phi = 2. * (velQuant + expDetuning) * (1 + kRat) * (*tPart) * gamToE;
        cx ephi = cx_make(cos(phi), sin(phi));  /* std::exp(complex(0,phi)) = polar(1,phi) */
        cx ham[NS][NS];
        memcpy(ham, s->hamCoupNoT, sizeof(ham));
        double a8 = ((p->OmDP / 2) * gs[8]) / sqrt(r);
        double a11 = ((p->OmDP / 2) * gs[11]) / sqrt(r);
        ham[8][5] = cx_sub(ham[8][5], cx_rscale(a8, ephi));   /* wvFn9*wvFn6.t() */
        ham[9][4] = cx_sub(ham[9][4], cx_rscale(a11, ephi));  /* wvFn10*wvFn5.t() */
        double E[NS] = {0};
        E[2] = totalDetRightSP; E[3] = totalDetRightSP;
        E[4] = totalDetLeftSP; E[5] = totalDetLeftSP;
        E[6] = (-p->detuning + p->detuningDP + (1 - kRat) * (velQuant + expDetuning));
        E[7] = E[6];
        E[10] = (-p->detuning + p->detuningDP + (kRat - 1) * (velQuant + expDetuning));
        E[11] = E[10];
        E[8] = (-p->detuning + p->detuningDP - velQuant - expDetuning - kRat * (velQuant + expDetuning));
        E[9] = E[8];
        cx hamil[NS][NS];
        for (int a = 0; a < NS; ++a)
            for (int b = 0; b < NS; ++b) {
                cx hE = cx_make(a == b ? E[a] : 0., 0.);
                cx h = cx_add(cx_add(hE, ham[a][b]), cx_conj(ham[b][a])); /* E + C + C^H */
                hamil[a][b] = cx_add(h, s->hamDecay[a][b]);                  /* + hamDecayTerm */
            }
        /* matPrefactor = ident - I*dtQuant*gamToE*hamil (:525-526) */
        double dtHalf = dtQuant * gamToE / 2;
        cx sI = cx_make(0., dtQuant * gamToE);
        cx M[NS][NS];
        for (int a = 0; a < NS; ++a)
            for (int b = 0; b < NS; ++b)
                M[a][b] = cx_sub(cx_make(a == b ? 1. : 0., 0.), cx_mul(sI, hamil[a][b]));
        const double h = dtQuant * gamToE;
        const double invh = 1. / (dtQuant * gamToE);
        cx y[NS], ws[NS], k1[NS], k2[NS], k3[NS], k4[NS], yk[NS];
        /* k1 (:530-536) */
        double pref = 1 / sqrt(1 - dp_of(s, wvFn, h));
        matvec(M, wvFn, ws);
        for (int k = 0; k < NS; ++k) {
            k1[k] = cx_rscale(invh, cx_sub(cx_rscale(pref, ws[k]), wvFn[k]));
            yk[k] = cx_add(wvFn[k], cx_rscale(dtHalf, k1[k]));
        }
        /* k2 (:541-546) */
        memcpy(y, yk, sizeof(y));
        pref = 1 / sqrt(1 - dp_of(s, y, h));
        matvec(M, y, ws);
        for (int k = 0; k < NS; ++k) {
            k2[k] = cx_rscale(invh, cx_sub(cx_rscale(pref, ws[k]), y[k]));
            yk[k] = cx_add(wvFn[k], cx_rscale(dtHalf, k2[k]));
        }
        /* k3 (:552-557) */
        memcpy(y, yk, sizeof(y));
        pref = 1 / sqrt(1 - dp_of(s, y, h));
        matvec(M, y, ws);
        for (int k = 0; k < NS; ++k) {
            k3[k] = cx_rscale(invh, cx_sub(cx_rscale(pref, ws[k]), y[k]));
            yk[k] = cx_add(wvFn[k], cx_rscale(h, k3[k]));
        }
        /* k4 (:562-567) */
        memcpy(y, yk, sizeof(y));
        pref = 1 / sqrt(1 - dp_of(s, y, h));
        matvec(M, y, ws);
        for (int k = 0; k < NS; ++k) {
            k4[k] = cx_rscale(invh, cx_sub(cx_rscale(pref, ws[k]), y[k]));
            cx sum = cx_add(cx_add(cx_add(k1[k], cx_rscale(3., k2[k])), cx_rscale(3., k3[k])), k4[k]);
            cx inc = cx_rscale(h, cx_make(sum.re / 8, sum.im / 8));
            wvFn[k] = cx_add(wvFn[k], inc);
        }
    } else {                                                                    /* :573-703 */
        jumped = 1;
        *tPart = 0;
        double rand2 = draw(g);
        double norm3 = cx_norm(wvFn[2]), norm4 = cx_norm(wvFn[3]);
        double norm5 = cx_norm(wvFn[4]), norm6 = cx_norm(wvFn[5]);
        double totalNorm = norm3 + norm4 + norm5 + norm6;
        double prob3 = norm3 / totalNorm, prob4 = norm4 / totalNorm, prob5 = norm5 / totalNorm;
        for (int k = 0; k < NS; ++k) wvFn[k] = cx_make(0., 0.);
        double randDOrS = draw(g);
        int sDecay = 1;
        double randDir = draw(g);
        if (randDOrS < (r / (r + 1))) {
            sDecay = 0;
            kick = (randDir < 0.5) ? s->vKickDP : -s->vKickDP;
        } else {
            kick = (randDir < 0.5) ? s->vKick : -s->vKick;
        }
        int target;
        if (rand2 < prob3) {
            if (sDecay) target = 1;
            else {
                double rand3 = draw(g);
                if (rand3 < gs[17] * gs[17] / r) target = 11;
                else if (rand3 < gs[17] * gs[17] / r + gs[16] * gs[16] / r) target = 10;
                else target = 9;
            }
        } else if (rand2 < prob3 + prob4) {
            double rand3 = draw(g);
            if (sDecay) target = (rand3 < gs[2] * gs[2]) ? 0 : 1;
            else {
                if (rand3 < gs[14] * gs[14] / r) target = 10;
                else if (rand3 < gs[14] * gs[14] / r + gs[13] * gs[13] / r) target = 9;
                else target = 8;
            }
        } else if (rand2 < prob3 + prob4 + prob5) {
            double rand3 = draw(g);
            if (sDecay) target = (rand3 < gs[4] * gs[4]) ? 1 : 0;
            else {
                if (rand3 < gs[11] * gs[11] / r) target = 9;
                else if (rand3 < gs[11] * gs[11] / r + gs[10] * gs[10] / r) target = 8;
                else target = 7;
            }
        } else {
            if (sDecay) target = 0;
            else {
                double rand3 = draw(g);
                if (rand3 < gs[8] * gs[8] / r) target = 8;
                else if (rand3 < gs[8] * gs[8] / r + gs[7] * gs[7] / r) target = 7;
                else target = 6;
            }
        }
        wvFn[target].re = 1;
    }
    *vx = *vx + kick;                                                           /* :705 */
    if (p->reNormalizewvFns) {                                                  /* :706-712 */
        double popS = cx_norm(wvFn[0]) + cx_norm(wvFn[1]);
        double popP = cx_norm(wvFn[2]) + cx_norm(wvFn[3]) + cx_norm(wvFn[4]) + cx_norm(wvFn[5]);
        double popD = cx_norm(wvFn[6]) + cx_norm(wvFn[7]) + cx_norm(wvFn[8]) + cx_norm(wvFn[9]) +
                      cx_norm(wvFn[10]) + cx_norm(wvFn[11]);
        double nrm = sqrt(popS + popP + popD);
        for (int k = 0; k < NS; ++k) wvFn[k] = cx_make(wvFn[k].re / nrm, wvFn[k].im / nrm);
    }
    for (int k = 0; k < NS; ++k) { psi[2 * k] = wvFn[k].re; psi[2 * k + 1] = wvFn[k].im; } /* :704 */
    return jumped;
}

/* ------------------------------------------------------------------------------------------ */
/* optical-pumping qstep (randomFrozenStartTag408Linear.cpp:396-598, 408Quad :399, 422Linear   */
/* :390-566; MonteCarloFollowedByQTTagging*.cpp :555): dense literal restatement               */
/* ------------------------------------------------------------------------------------------ */

typedef struct { int nst, nch, ncp; int a[10], b[10]; double g[10]; int ca[4], cb[4], cg[4]; } pump_model;

/* cs[j] = |a_j><b_j|, gs[j] (408 main :1000-1019; 422 main), couplings (:438) */
static void pump_model_of(int m, double r, pump_model* pm) {
    static const int A408[10] = {0, 0, 0, 1, 1, 1, 6, 6, 6, 6}, B408[10] = {2, 3, 4, 3, 4, 5, 2, 3, 4, 5};
    static const int A422[6] = {1, 1, 0, 0, 4, 4}, B422[6] = {2, 3, 3, 2, 2, 3};
    memset(pm, 0, sizeof(*pm));
    if (m == 3) {
        const double G[6] = {2. / 3, 1. / 3, 2. / 3, 1. / 3, r, r};
        pm->nst = 5; pm->nch = 6;
        for (int j = 0; j < 6; ++j) { pm->a[j] = A422[j]; pm->b[j] = B422[j]; pm->g[j] = G[j]; }
        /* -Om/2 wvFn2 wvFn3^H sqrt(gs[0]) - Om/2 wvFn1 wvFn4^H sqrt(gs[2]) (422Linear :97) */
        pm->ncp = 2; pm->ca[0] = 1; pm->cb[0] = 2; pm->cg[0] = 0; pm->ca[1] = 0; pm->cb[1] = 3; pm->cg[1] = 2;
    } else {
        const double G[10] = {1, 2. / 3, 1. / 3, 1. / 3, 2. / 3, 1, r, r, r, r};
        pm->nst = 7; pm->nch = 10;
        for (int j = 0; j < 10; ++j) { pm->a[j] = A408[j]; pm->b[j] = B408[j]; pm->g[j] = G[j]; }
        if (m == 1) {   /* wvFn2 wvFn4^H gs3, wvFn2 wvFn6^H gs5, wvFn1 wvFn3^H gs0, wvFn1 wvFn5^H gs2 */
            pm->ncp = 4;
            pm->ca[0] = 1; pm->cb[0] = 3; pm->cg[0] = 3;
            pm->ca[1] = 1; pm->cb[1] = 5; pm->cg[1] = 5;
            pm->ca[2] = 0; pm->cb[2] = 2; pm->cg[2] = 0;
            pm->ca[3] = 0; pm->cb[3] = 4; pm->cg[3] = 2;
        } else {        /* 408Quad: wvFn2 wvFn6^H gs5, wvFn1 wvFn5^H gs2 */
            pm->ncp = 2;
            pm->ca[0] = 1; pm->cb[0] = 5; pm->cg[0] = 5;
            pm->ca[1] = 0; pm->cb[1] = 4; pm->cg[1] = 2;
        }
    }
}

/* dpmat = sum_j (c * y^H cs_j^H cs_j y) * gs[j] (:419-425); cs_j^H cs_j = |b_j><b_j| */
static double pump_dp(const pump_model* pm, const cx* y, double c) {
    double dp = 0.;
    for (int j = 0; j < pm->nch; ++j) {
        const cx yb = y[pm->b[j]];
        dp = dp + (c * cx_mul(cx_conj(yb), yb).re) * pm->g[j];
    }
    return dp;
}

static int qstep_ion_pump(const orc_sim* s, double* psi, double* vx, double* tPart, rngsrc* g) {
    const orc_params* p = &s->p;
    const int m = p->qt_model;
    pump_model pm;
    pump_model_of(m, s->r, &pm);
    const int nP = m == 3 ? 2 : 4;
    const double dtQuant = s->dtQ, gamToE = s->gamToE;
    const double h = dtQuant * gamToE;
    cx wvFn[NS];
    for (int k = 0; k < NS; ++k) wvFn[k] = cx_make(psi[2 * k], psi[2 * k + 1]);
    const double velQuant = (*vx) * s->plasVelToQuantVel;                       /* :407-408 */
    *tPart += dtQuant;   /* engine bookkeeping only: the pumping H has no time-dependent term */
    const double dp = pump_dp(&pm, wvFn, h);                                    /* :419-425 */
    const double rand = draw(g);                                                /* :426 */
    int jumped = 0;
    if (rand > dp) {
        const double totalDetRightSP = -p->detuning - velQuant;                 /* :436 */
        const double totalDetLeftSP = -p->detuning + velQuant;                  /* :437 */
        cx C[NS][NS];
        memset(C, 0, sizeof(C));
        for (int c = 0; c < pm.ncp; ++c)                                        /* :438 */
            C[pm.ca[c]][pm.cb[c]] = cx_add(C[pm.ca[c]][pm.cb[c]], cx_make((-p->Om / 2) * sqrt(pm.g[pm.cg[c]]), 0.));
        double E[NS] = {0};                                                     /* :439 */
        for (int k = 2; k < 2 + nP; ++k) E[k] = (k < 2 + nP / 2) ? totalDetRightSP : totalDetLeftSP;
        double Dd[NS] = {0};                                                    /* :444-447 */
        for (int j = 0; j < pm.nch; ++j) Dd[pm.b[j]] = Dd[pm.b[j]] + pm.g[j];
        cx M[NS][NS];
        const cx sI = cx_make(0., h);
        for (int a = 0; a < NS; ++a)
            for (int b = 0; b < NS; ++b) {
                cx hm = cx_add(cx_add(cx_make(a == b ? E[a] : 0., 0.), C[a][b]), cx_conj(C[b][a]));
                if (a == b) hm = cx_add(hm, cx_make(0., -0.5 * Dd[a]));          /* hamDecayTerm */
                M[a][b] = cx_sub(cx_make(a == b ? 1. : 0., 0.), cx_mul(sI, hm));  /* :465 */
            }
        const double dtHalf = h / 2, invh = 1. / h;
        cx y[NS], ws[NS], k1[NS], k2[NS], k3[NS], k4[NS], yk[NS];
        double pref = 1 / sqrt(1 - pump_dp(&pm, wvFn, h));                    /* :457-468 */
        matvec(M, wvFn, ws);
        for (int k = 0; k < NS; ++k) {
            k1[k] = cx_rscale(invh, cx_sub(cx_rscale(pref, ws[k]), wvFn[k]));
            yk[k] = cx_add(wvFn[k], cx_rscale(dtHalf, k1[k]));
        }
        memcpy(y, yk, sizeof(y));                                               /* :471-481 */
        pref = 1 / sqrt(1 - pump_dp(&pm, y, h));
        matvec(M, y, ws);
        for (int k = 0; k < NS; ++k) {
            k2[k] = cx_rscale(invh, cx_sub(cx_rscale(pref, ws[k]), y[k]));
            yk[k] = cx_add(wvFn[k], cx_rscale(dtHalf, k2[k]));
        }
        memcpy(y, yk, sizeof(y));                                               /* :486-496 */
        pref = 1 / sqrt(1 - pump_dp(&pm, y, h));
        matvec(M, y, ws);
        for (int k = 0; k < NS; ++k) {
            k3[k] = cx_rscale(invh, cx_sub(cx_rscale(pref, ws[k]), y[k]));
            yk[k] = cx_add(wvFn[k], cx_rscale(h, k3[k]));
        }
        memcpy(y, yk, sizeof(y));                                               /* :500-510 */
        pref = 1 / sqrt(1 - pump_dp(&pm, y, h));
        matvec(M, y, ws);
        for (int k = 0; k < NS; ++k) k4[k] = cx_rscale(invh, cx_sub(cx_rscale(pref, ws[k]), y[k]));
        for (int k = 0; k < NS; ++k) {                                          /* :511 */
            cx sum = cx_add(cx_add(cx_add(k1[k], cx_rscale(3., k2[k])), cx_rscale(3., k3[k])), k4[k]);
            wvFn[k] = cx_add(wvFn[k], cx_rscale(h, cx_rscale(1. / 8, sum)));
        }
    } else {                                                                    /* :513-596 */
        jumped = 1;
        *tPart = 0;
        const double rand2 = draw(g);
        const double n3 = cx_norm(wvFn[2]), n4 = cx_norm(wvFn[3]);
        const double n5 = cx_norm(wvFn[4]), n6 = cx_norm(wvFn[5]);
        for (int k = 0; k < NS; ++k) wvFn[k] = cx_make(0., 0.);
        int target;
        const double randDOrS = draw(g);
        const int sDecay = !(randDOrS < (s->r / (s->r + 1)));
        if (m == 3) {                                           /* 422Linear :174-231 */
            const double totalNorm = n3 + n4, prob3 = n3 / totalNorm;
            if (rand2 < prob3) target = sDecay ? ((draw(g) < 2. / 3) ? 1 : 0) : 4;
            else target = sDecay ? ((draw(g) < 2. / 3) ? 0 : 1) : 4;
        } else {                                                /* 408 :513-590 */
            const double totalNorm = n3 + n4 + n5 + n6;
            const double prob3 = n3 / totalNorm, prob4 = n4 / totalNorm, prob5 = n5 / totalNorm;
            (void)draw(g);                                      /* randDir (unused) */
            if (rand2 < prob3) target = sDecay ? 0 : 6;
            else if (rand2 < prob3 + prob4) target = sDecay ? ((draw(g) < 2. / 3) ? 0 : 1) : 6;
            else if (rand2 < prob3 + prob4 + prob5) target = sDecay ? ((draw(g) < 1. / 3) ? 0 : 1) : 6;
            else target = sDecay ? 1 : 6;
        }
        wvFn[target] = cx_make(1., 0.);
    }
    (void)pm.a;
    for (int k = 0; k < NS; ++k) { psi[2 * k] = wvFn[k].re; psi[2 * k + 1] = wvFn[k].im; }
    return jumped;
}

int orc_tag_spin_up(const orc_sim* s, int* tags) {
    const int m = s->p.qt_model;
    if (m == 0) return -1;
    int cnt = 0;
    for (int i = 0; i < s->N; ++i) {
        const double* w = s->psi + (size_t)24 * i;
        double nr[5];
        for (int k = 0; k < 5; ++k) nr[k] = w[2 * k] * w[2 * k] + w[2 * k + 1] * w[2 * k + 1];
        const double rnd = orc_philox_uniform(s->p.seed, s->p.job, (uint64_t)i, s->qidx, 6);
        const double r2 = orc_philox_uniform(s->p.seed, s->p.job, (uint64_t)i, s->qidx, 7);
        int up;
        if (m == 3) {                                           /* 422Linear :568-600 */
            if (rnd < nr[0]) up = 1;
            else if (rnd < nr[0] + nr[2]) up = r2 < 1. / 3;
            else if (rnd < nr[0] + nr[2] + nr[3]) up = r2 < 2. / 3;
            else up = 0;
        } else {                                                /* 408Linear :600-640 */
            if (rnd < nr[0] + nr[2]) up = 1;
            else if (rnd < nr[0] + nr[2] + nr[3]) up = r2 < 2. / 3;
            else if (rnd < nr[0] + nr[2] + nr[3] + nr[4]) up = r2 < 1. / 3;
            else up = 0;
        }
        if (tags) tags[i] = up;
        cnt += up;
    }
    return cnt;
}

int orc_qstep_ion(const orc_sim* s, double t, double* psi, double* vx, double* tPart,
                  const double u[5], int* ndraws) {
    rngsrc g; memset(&g, 0, sizeof(g));
    g.mode = 2; g.tape = u;
    int j = s->p.qt_model != 0 ? qstep_ion_pump(s, psi, vx, tPart, &g)
                               : qstep_ion(s, t, expDetuning_of(s, t), psi, vx, tPart, &g);
    if (ndraws) *ndraws = g.n;
    return j;
}

void orc_qstep(orc_sim* s) {
    if (s->p.qt_enabled) {
        double expDet = expDetuning_of(s, s->t);
        int c = s->cap;
        if (s->p.rng_mode == 0) {
            /* drand48: one shared stream consumed in ion order (1-thread reference) */
            rngsrc g; memset(&g, 0, sizeof(g));
            g.mode = 0; g.x48 = &s->x48;
            for (int i = 0; i < s->N; i++) {
                if (s->p.qt_model != 0) qstep_ion_pump(s, s->psi + (size_t)24 * i, &s->V[i], &s->tPart[i], &g);
                else qstep_ion(s, s->t, expDet, s->psi + (size_t)24 * i, &s->V[i], &s->tPart[i], &g);
            }
        } else {
#ifdef _OPENMP
#pragma omp parallel for schedule(static) num_threads(s->p.nthreads > 0 ? s->p.nthreads : 1)
#endif
            for (int i = 0; i < s->N; i++) {
                rngsrc g; memset(&g, 0, sizeof(g));
                g.mode = 1; g.seed = s->p.seed; g.job = s->p.job; g.qidx = s->qidx;
                g.ion = (s->ion_ids && i < s->n_ion_ids) ? s->ion_ids[i] : (uint64_t)i;
                if (s->p.qt_model != 0) qstep_ion_pump(s, s->psi + (size_t)24 * i, &s->V[i], &s->tPart[i], &g);
                else qstep_ion(s, s->t, expDet, s->psi + (size_t)24 * i, &s->V[i], &s->tPart[i], &g);
            }
        }
        (void)c;
    }
    s->qidx++;
    s->t += s->dtQ;                                                             /* :716 */
}

void orc_substeps(orc_sim* s, int n) {
    for (int k = 0; k < n; ++k) { orc_step(s); orc_qstep(s); }
}

void orc_md_steps(orc_sim* s, int n) {
    for (int k = 0; k < n; ++k) {
        orc_forces(s);
        s->c0++;
        orc_substeps(s, s->ratio);
    }
}

/* ------------------------------------------------------------------------------------------ */
/* output (SpeedUp:917-1032)                                                                     */
/* ------------------------------------------------------------------------------------------ */

void orc_observables(orc_sim* s, double out7[7], double* Pvel, double* pops) {
    int N = s->N, c = s->cap;
    const double *Vx = s->V, *Vy = s->V + c, *Vz = s->V + 2 * c;
    double velXAvg = 0.0, EkinX = 0.0, EkinY = 0.0, EkinZ = 0.0;
    for (int i = 0; i < N; i++) velXAvg += Vx[i];                              /* :934-938 */
    velXAvg /= (double)N;
    for (int i = 0; i < N; i++) {                                               /* :939-944 */
        EkinX += 0.5 * ((Vx[i] - velXAvg) * (Vx[i] - velXAvg));
        EkinY += 0.5 * (Vy[i] * Vy[i]);
        EkinZ += 0.5 * (Vz[i] * Vz[i]);
    }
    EkinX /= (double)N; EkinY /= (double)N; EkinZ /= (double)N;
    orc_epotential(s);                                                          /* :948 */
    out7[0] = s->t; out7[1] = EkinX; out7[2] = EkinY; out7[3] = EkinZ; out7[4] = s->Epot;
    out7[5] = EkinX + EkinY + EkinZ + s->Epot - s->Epot0; out7[6] = velXAvg;    /* :954 */
    if (Pvel) {                                                                 /* :957-979 */
        double V2 = 1. / (2. * 0.002 * 0.002);
        double *PX = Pvel, *PY = Pvel + NBINS, *PZ = Pvel + 2 * NBINS;
        const double* vel = s->vel;
        for (int j = 0; j < NBINS; j++) { PX[j] = 0.0; PY[j] = 0.0; PZ[j] = 0.0; }
        for (int i = 0; i < N; i++) {
            for (int j = 0; j < NBINS; j++) {
                PX[j] += exp(-V2 * (vel[j] - (Vx[i] - velXAvg)) * (vel[j] - (Vx[i] - velXAvg))) +
                         exp(-V2 * (vel[j] + (Vx[i] - velXAvg)) * (vel[j] + (Vx[i] - velXAvg)));
                PY[j] += exp(-V2 * (vel[j] - Vy[i]) * (vel[j] - Vy[i])) + exp(-V2 * (vel[j] + Vy[i]) * (vel[j] + Vy[i]));
                PZ[j] += exp(-V2 * (vel[j] - Vz[i]) * (vel[j] - Vz[i])) + exp(-V2 * (vel[j] + Vz[i]) * (vel[j] + Vz[i]));
            }
        }
        for (int j = 0; j < NBINS; j++) {
            PX[j] /= (6.0 * sqrt(2 * M_PI * 0.002 * 0.002));
            PY[j] /= (6.0 * sqrt(2 * M_PI * 0.002 * 0.002));
            PZ[j] /= (6.0 * sqrt(2 * M_PI * 0.002 * 0.002));
        }
    }
    if (pops) {                                                                 /* :1016-1023 */
        for (int i = 0; i < N; i++) {
            cx w[NS];
            const double* ps = s->psi + (size_t)24 * i;
            for (int k = 0; k < NS; ++k) w[k] = cx_make(ps[2 * k], ps[2 * k + 1]);
            pops[3 * i + 0] = cx_norm(w[0]) + cx_norm(w[1]);
            pops[3 * i + 1] = cx_norm(w[2]) + cx_norm(w[3]) + cx_norm(w[4]) + cx_norm(w[5]);
            pops[3 * i + 2] = cx_norm(w[6]) + cx_norm(w[7]) + cx_norm(w[8]) + cx_norm(w[9]) +
                              cx_norm(w[10]) + cx_norm(w[11]);
        }
    }
}

static FILE* open_in(const orc_sim* s, const char* name, const char* mode) {
    char path[1024];
    snprintf(path, sizeof(path), "%s%s", s->saveDirectory, name);
    FILE* f = fopen(path, mode);
    if (!f) fprintf(stderr, "oracle: cannot open %s: %s\n", path, strerror(errno));
    return f;
}

int orc_output(orc_sim* s) {
    double o[7];
    double* P = malloc(sizeof(double) * 3 * NBINS);
    double* pops = malloc(sizeof(double) * 3 * (size_t)(s->N > 0 ? s->N : 1));
    if (!P || !pops) { free(P); free(pops); return -1; }
    orc_observables(s, o, P, pops);
    FILE* fa = open_in(s, "energies.dat", "a");
    if (!fa) { free(P); free(pops); return -1; }
    fprintf(fa, "%lg\t%lg\t%lg\t%lg\t%lg\t%lg\t%lg\n", o[0], o[1], o[2], o[3], o[4], o[5], o[6]);
    fclose(fa);
    char b1[64], b2[64], b3[64];
    snprintf(b1, sizeof b1, "vel_distX_time%06d.dat", s->counter);
    snprintf(b2, sizeof b2, "vel_distY_time%06d.dat", s->counter);
    snprintf(b3, sizeof b3, "vel_distZ_time%06d.dat", s->counter);
    FILE *f1 = open_in(s, b1, "w"), *f2 = open_in(s, b2, "w"), *f3 = open_in(s, b3, "w");
    if (!f1 || !f2 || !f3) { if (f1) fclose(f1); if (f2) fclose(f2); if (f3) fclose(f3); free(P); free(pops); return -1; }
    for (int i = 0; i < NBINS; i++) {
        fprintf(f1, "%lg\t%lg\n", s->vel[i] + o[6], P[i]);
        fprintf(f2, "%lg\t%lg\n", s->vel[i], P[NBINS + i]);
        fprintf(f3, "%lg\t%lg\n", s->vel[i], P[2 * NBINS + i]);
    }
    fclose(f1); fclose(f2); fclose(f3);
    snprintf(b1, sizeof b1, "statePopulationsVsVTime%06d.dat", s->counter);
    fa = open_in(s, b1, "w");
    if (!fa) { free(P); free(pops); return -1; }
    for (int i = 0; i < s->N; i++)
        fprintf(fa, "%lg\t%lg\t%lg\t%lg\n", s->V[i], pops[3 * i], pops[3 * i + 1], pops[3 * i + 2]);
    fclose(fa);
    s->counter++;                                                               /* :1027 */
    free(P); free(pops);
    return 0;
}

int orc_write_conditions(orc_sim* s, int c0) {                                 /* :725-784 */
    char b[96];
    int N = s->N, c = s->cap;
    snprintf(b, sizeof b, "ions_timestep%06d.dat", c0);
    FILE* fa = open_in(s, b, "w");
    if (!fa) return -1;
    fprintf(fa, "%i\t%i", N, s->counter);
    fclose(fa);
    snprintf(b, sizeof b, "conditions_timestep%06d.dat", c0);
    fa = open_in(s, b, "w");
    if (!fa) return -1;
    for (int i = 0; i < N; i++)
        fprintf(fa, "%lg\t%lg\t%lg\t%lg\t%lg\t%lg\t\n", s->R[i], s->R[c + i], s->R[2 * c + i], s->V[i],
                s->V[c + i], s->V[2 * c + i]);
    fclose(fa);
    for (int v = 0; v < NINTERVALV; v++) {
        snprintf(b, sizeof b, "VZERO_timestep%06d_interval%d.dat", c0, v);
        fa = open_in(s, b, "w");
        if (!fa) return -1;
        const double* vh = s->Vholder + (size_t)v * 3 * c;
        for (int i = 0; i < N; i++) fprintf(fa, "%lg\t%lg\t%lg\n", vh[i], vh[c + i], vh[2 * c + i]);
        fclose(fa);
    }
    snprintf(b, sizeof b, "wvFns_timestep%06d.dat", c0);
    fa = open_in(s, b, "w");
    if (!fa) return -1;
    for (int j = 0; j < N; j++) {
        const double* ps = s->psi + (size_t)24 * j;
        for (int k = 0; k < NS; k++) fprintf(fa, "%lg\t%lg\t", ps[2 * k], ps[2 * k + 1]);
        fprintf(fa, "\n");
    }
    fclose(fa);
    return 0;
}

int orc_read_conditions(orc_sim* s, int c0) {                                  /* :785-916 */
    s->t = ((double)c0 - 9.) * TIMESTEP + 0.02;
    char b[96];
    snprintf(b, sizeof b, "ions_timestep%06d.dat", c0);
    FILE* fa = open_in(s, b, "r");
    if (!fa) return -1;
    int j, m;
    while (fscanf(fa, "%i\t%i", &j, &m) == 2) { s->N = j; s->counter = (unsigned)m; }
    fclose(fa);
    if (s->N + 64 > s->cap && reserve(s, s->N + 64)) return -1;
    int c = s->cap;
    snprintf(b, sizeof b, "conditions_timestep%06d.dat", c0);
    fa = open_in(s, b, "r");
    if (!fa) return -1;
    double a, bb, z, d, e, f;
    int i = 0;
    while (i < s->N && fscanf(fa, "%lg\t%lg\t%lg\t%lg\t%lg\t%lg\n", &a, &bb, &z, &d, &e, &f) == 6) {
        s->R[i] = a; s->R[c + i] = bb; s->R[2 * c + i] = z;
        s->V[i] = d; s->V[c + i] = e; s->V[2 * c + i] = f;
        i++;
    }
    fclose(fa);
    snprintf(b, sizeof b, "wvFns_timestep%06d.dat", c0);
    fa = open_in(s, b, "r");
    if (!fa) return -1;
    i = 0;
    double w[24];
    while (i < s->N &&
           fscanf(fa, "%lg%lg\t%lg%lg\t%lg%lg\t%lg%lg\t%lg%lg\t%lg%lg\t%lg%lg\t%lg%lg\t%lg%lg\t%lg%lg\t%lg%lg\t%lg%lg\n",
                  &w[0], &w[1], &w[2], &w[3], &w[4], &w[5], &w[6], &w[7], &w[8], &w[9], &w[10], &w[11], &w[12],
                  &w[13], &w[14], &w[15], &w[16], &w[17], &w[18], &w[19], &w[20], &w[21], &w[22], &w[23]) == 24) {
        memcpy(s->psi + (size_t)24 * i, w, sizeof(w));
        i++;
    }
    fclose(fa);
    for (int v = 0; v < NINTERVALV; v++) {
        snprintf(b, sizeof b, "VZERO_timestep%06d_interval%d.dat", c0, v);
        fa = open_in(s, b, "r");
        if (!fa) return -1;
        double* vh = s->Vholder + (size_t)v * 3 * c;
        i = 0;
        while (i < s->N && fscanf(fa, "%lg\t%lg\t%lg", &a, &bb, &z) == 3) {
            vh[i] = a; vh[c + i] = bb; vh[2 * c + i] = z;
            i++;
        }
        fclose(fa);
    }
    /* tPart and Epot0 are not restored by the reference */
    s->c0 = c0;
    s->qidx = (uint64_t)(c0 + 1) * (uint64_t)s->ratio;
    return 0;
}

/* the reference's "(unsigned)(x)" printed with %d: a truncating conversion through 64-bit
 * int, low 32 bits reinterpreted as signed (x86-64 runtime behaviour) */
static int ref_udcast(double x) { return (int)(uint32_t)(int64_t)x; }

int orc_setup_directories(orc_sim* s) {                                       /* :1145-1160 */
    const orc_params* p = &s->p;
    char base[512];
    strncpy(base, p->saveDirectory, sizeof(base) - 1);
    base[sizeof(base) - 1] = 0;
    mkdir(base, 0777);
    char name[256];
    snprintf(name, sizeof name, "Ge%dDensity%dE+11Sig0%dTe%dSigFrac%dDetSP%dDetDP%dOmSP%dOmDP%dNumIons%d",
             ref_udcast(100 * p->Ge), ref_udcast(p->density * 1000), ref_udcast(10 * p->sig0), ref_udcast(p->Te),
             ref_udcast(p->fracOfSig * 100), ref_udcast(p->detuning * 100), ref_udcast(p->detuningDP * 100),
             ref_udcast(p->Om * 100), ref_udcast(p->OmDP * 100), ref_udcast((double)p->N0));
    snprintf(s->saveDirectory, sizeof(s->saveDirectory), "%s%s", base, name);
    mkdir(s->saveDirectory, 0777);
    char jb[64];
    snprintf(jb, sizeof jb, "/job%d/", (int)p->job);
    strncat(s->saveDirectory, jb, sizeof(s->saveDirectory) - strlen(s->saveDirectory) - 1);
    mkdir(s->saveDirectory, 0777);
    return 0;
}

int orc_run(orc_sim* s) {                                                      /* :1139-1383 */
    if (orc_setup_directories(s)) return -1;
    s->x48 = orc_srand48_state(s->p.seed);
    if (s->p.newRun == 1) {
        if (orc_init(s)) return -1;
    } else {
        s->c0 = s->p.c0;
        if (orc_read_conditions(s, s->c0)) return -1;
    }
    int timeStepCounter = s->ratio;                                           /* :1235 */
    while (s->t <= s->p.tmax + 0.0009) {                                       /* :1248 */
        if ((s->c0 + 1) % s->p.sampleFreq == 0 && timeStepCounter == 1) {      /* :1365 */
            if (orc_output(s)) return -1;
        }
        if (timeStepCounter == s->ratio) {                                     /* :1369 */
            orc_forces(s);
            s->c0++;
            timeStepCounter = 0;
        }
        orc_step(s);
        orc_qstep(s);
        timeStepCounter++;
    }
    return orc_write_conditions(s, s->c0);                                    /* :1381 */
}

/* ------------------------------------------------------------------------------------------ */
/* The optical-pumping programs' main(): randomFrozenStartTag408Linear.cpp (":" lines),         */
/* randomFrozenStartTag408Quad.cpp and randomFrozenStartTag422Linear.cpp follow the same flow.   */
/* ------------------------------------------------------------------------------------------ */

static void step_R_pump(orc_sim* s, double DT) {                                 /* :317-356 */
    const int c = s->cap;
    if (s->t > 0) {
        for (int i = 0; i < s->N; i++)
            for (int k = 0; k < 3; ++k) s->R[(size_t)k * c + i] += DT * s->V[(size_t)k * c + i];
    } else {
        orc_forces(s);
        for (int i = 0; i < s->N; i++)
            for (int k = 0; k < 3; ++k)
                s->R[(size_t)k * c + i] += DT * s->V[(size_t)k * c + i] + DT * DT * s->F[(size_t)k * c + i];
    }
    for (int i = 0; i < s->N; i++)
        for (int k = 0; k < 3; ++k) {
            double* r = &s->R[(size_t)k * c + i];
            if (*r < 0) *r += s->L;
            if (*r > s->L) *r -= s->L;
        }
}

static void md_step_pump(orc_sim* s) {                                           /* :377-394 */
    const int c = s->cap;
    const double dt = s->dtQ * s->ratio;
    step_R_pump(s, 0.5 * dt);
    orc_forces(s);                                                               /* step_V :358-375 */
    for (int i = 0; i < s->N; i++)
        for (int k = 0; k < 3; ++k) s->V[(size_t)k * c + i] += dt * s->F[(size_t)k * c + i];
    step_R_pump(s, 0.5 * dt);
}

static int setup_dirs_pump(orc_sim* s) {                                         /* :985-999 */
    const orc_params* p = &s->p;
    char base[512];
    strncpy(base, p->saveDirectory, sizeof(base) - 1);
    base[sizeof(base) - 1] = 0;
    mkdir(base, 0777);
    char name[256];
    snprintf(name, sizeof name, "PumpTime%dPumpStart%dDet%dOm%dDensity%dGe%dNumIons%d",
             (int)(unsigned)(1000000000. * p->tpumpreal), (int)(unsigned)(p->tstartV0),
             (int)(unsigned)(100. * fabs(p->detuning)), (int)(unsigned)(100. * p->Om),
             (int)(unsigned)(10. * p->density), (int)(unsigned)(1000 * p->Ge), (int)(unsigned)p->N0);
    snprintf(s->saveDirectory, sizeof(s->saveDirectory), "%s%s", base, name);
    mkdir(s->saveDirectory, 0777);
    char jb[64];
    snprintf(jb, sizeof jb, "/job%d/", (int)p->job);
    strncat(s->saveDirectory, jb, sizeof(s->saveDirectory) - strlen(s->saveDirectory) - 1);
    mkdir(s->saveDirectory, 0777);
    return 0;
}

static int measure_spin_ups_pump(orc_sim* s) {                                    /* :600-665 */
    free(s->spinUp);
    s->spinUp = calloc((size_t)(s->N > 0 ? s->N : 1), sizeof(int));
    s->nSpinUp = orc_tag_spin_up(s, s->spinUp);
    char b[96];
    snprintf(b, sizeof b, "spinUpIons_timestep%06d.dat", s->c0);
    FILE* fa = open_in(s, b, "w");
    if (!fa) return -1;
    fprintf(fa, "%i", s->nSpinUp);
    fclose(fa);
    return 0;
}

static int output_pump(orc_sim* s, int bin0) {                                    /* :799-935 */
    const int N = s->N, c = s->cap;
    const double *Vx = s->V, *Vy = s->V + c, *Vz = s->V + 2 * c;
    double EkinX = 0.0, EkinY = 0.0, EkinZ = 0.0;
    for (int i = 0; i < N; i++) {
        EkinX += 0.5 * (Vx[i] * Vx[i]);
        EkinY += 0.5 * (Vy[i] * Vy[i]);
        EkinZ += 0.5 * (Vz[i] * Vz[i]);
    }
    EkinX /= (double)N; EkinY /= (double)N; EkinZ /= (double)N;
    orc_epotential(s);
    FILE* fa = open_in(s, "energies.dat", "a");
    if (!fa) return -1;
    fprintf(fa, "%lg\t%lg\t%lg\t%lg\t%lg\t%lg\n", s->t, EkinX, EkinY, EkinZ, s->Epot, EkinX + EkinY + EkinZ + s->Epot - s->Epot0);
    fclose(fa);
    const double V2 = 1. / (2. * 0.002 * 0.002);
    double* PvelX = calloc(4001, sizeof(double));
    double firstMom = 0, secondMom = 0, thirdMom = 0, fourthMom = 0;
    unsigned numTagged = 0;
    for (int i = 0; i < N; i++) {
        const double currVx = Vx[i];
        const int up = s->spinUp ? s->spinUp[i] : 0;
        if (up) {
            firstMom += currVx; secondMom += currVx * currVx; thirdMom += currVx * currVx * currVx;
            fourthMom += currVx * currVx * currVx * currVx;
            numTagged += 1;
        }
        if (up == 1)
            for (int j = 0; j < 4001; j++) {
                const double vel = (double)(j + bin0) * 0.0025;
                PvelX[j] += exp(-V2 * (vel - Vx[i]) * (vel - Vx[i]));
            }
    }
    firstMom /= numTagged; secondMom /= numTagged; thirdMom /= numTagged; fourthMom /= numTagged;
    fa = open_in(s, "taggedMoments.dat", "a");
    if (!fa) { free(PvelX); return -1; }
    fprintf(fa, "%lg\t%lg\t%lg\t%lg\t%lg\n", s->t, firstMom, secondMom, thirdMom, fourthMom);
    fclose(fa);
    for (int j = 0; j < 4001; j++) PvelX[j] /= (6.0 * sqrt(2 * M_PI * 0.002 * 0.002));
    char b[96];
    snprintf(b, sizeof b, "vel_distX_timestep%06d.dat", s->c0);
    fa = open_in(s, b, "w");
    if (!fa) { free(PvelX); return -1; }
    for (int j = 0; j < 4001; j++) fprintf(fa, "%lg\t%lg\n", (double)(j + bin0) * 0.0025, PvelX[j]);
    fclose(fa);
    free(PvelX);
    s->counter++;
    return 0;
}

static int vaf_pump(orc_sim* s, int c1V) {                                        /* :938-975 */
    const int N = s->N;
    if (c1V == 0) {
        free(s->vaHold);
        s->vaHold = malloc(sizeof(double) * (size_t)(N > 0 ? N : 1));
        for (int j = 0; j < N; j++) s->vaHold[j] = s->V[j];
    }
    double VAF = 0.0;
    for (int j = 0; j < N; j++) VAF += 1 / ((double)(N)) * (s->vaHold[j] * s->V[j]);
    FILE* fa = open_in(s, "VAF.dat", "a");
    if (!fa) return -1;
    fprintf(fa, "%lg\t%lg\n", s->t, VAF);
    fclose(fa);
    return 0;
}

static int write_conditions_pump(orc_sim* s, int c0) {                           /* :667-707 */
    const int N = s->N, c = s->cap;
    char b[96];
    snprintf(b, sizeof b, "ions_timestep%06d.dat", c0);
    FILE* fa = open_in(s, b, "w");
    if (!fa) return -1;
    fprintf(fa, "%i\t%i", N, s->counter);
    fclose(fa);
    snprintf(b, sizeof b, "spinUpIonsList_timestep%06d.dat", c0);
    fa = open_in(s, b, "w");
    if (!fa) return -1;
    for (int i = 0; i < N; i++) fprintf(fa, "%i\n", s->spinUp ? s->spinUp[i] : 0);
    fclose(fa);
    snprintf(b, sizeof b, "conditions_timestep%06d.dat", c0);
    fa = open_in(s, b, "w");
    if (!fa) return -1;
    for (int i = 0; i < N; i++)
        fprintf(fa, "%lg\t%lg\t%lg\t%lg\t%lg\t%lg\t\n", s->R[i], s->R[c + i], s->R[2 * (size_t)c + i], s->V[i],
                s->V[c + i], s->V[2 * (size_t)c + i]);
    fclose(fa);
    return 0;
}

int orc_get_spin_up_list(const orc_sim* s, int* tags) {
    for (int i = 0; i < s->N && tags; ++i) tags[i] = s->spinUp ? s->spinUp[i] : 0;
    return s->nSpinUp;
}

int orc_run_pump(orc_sim* s) {                                                   /* :981-1076 */
    if (s->p.qt_model < 1 || s->p.qt_model > 3) return -1;
    if (setup_dirs_pump(s)) return -1;
    s->x48 = orc_srand48_state(s->p.seed);
    if (orc_init(s)) return -1;                                                  /* newRun == 1 */
    int recorded = 0;
    const int bin0 = -2000;                                                      /* init() :306 */
    const double tpump = s->p.tpumpreal * 813490 * sqrt(s->p.density);          /* :79 */
    const double tendV0 = s->p.tstartV0 + tpump;                                /* :80 */
    int tsc = s->ratio;                                                          /* :1033 */
    while (s->t <= s->p.tmax + 0.0009) {                                         /* :1050 */
        if (recorded == 0 && s->t >= tendV0) {                                   /* :1052-1058 */
            if (measure_spin_ups_pump(s)) return -1;
            recorded = 1;
            if (output_pump(s, bin0)) return -1;
            if (vaf_pump(s, 0)) return -1;
        }
        if ((s->c0 + 1) % s->p.sampleFreq == 0 && tsc == 1 && recorded == 1) {   /* :1062-1069 */
            if (output_pump(s, bin0)) return -1;
            if (vaf_pump(s, 1)) return -1;
        }
        if (tsc == s->ratio) {                                                   /* :1070-1074 */
            md_step_pump(s);
            s->c0++;
            tsc = 0;
        }
        if (s->t < tendV0 && s->t > s->p.tstartV0) orc_qstep(s);                /* :1075-1080 */
        else s->t += s->dtQ;
        tsc++;
    }
    return write_conditions_pump(s, s->c0);
}
