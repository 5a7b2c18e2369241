// The reference-side binding of INTEGRATION.md, compiled and driven.
//
// This program has the shape of laserCoolingPlusExpansionMDQTSpeedUp.cpp ("SpeedUp"): its user
// inputs and state as globals (SpeedUp:56-85, :111-160), the hot-path functions as `void f(void)`
// (prototypes SpeedUp:176-185) and main()'s time loop (SpeedUp:1139-1383) calling them in the
// reference's order.  The function bodies are the INTEGRATION.md stubs into libmdqt (include/mdqt.h);
// init() keeps the reference's own host sampling (restated here from SpeedUp:289-348, since the
// reference's source does not travel) and ends with push_state() + push_counters(), the two lines a
// maintainer appends.  main() gains one line, mdqt_attach(job), before saveDirectory is extended.
//
//   binding_check <job> <saveDirectory/> <N0> <tmax> <sampleFreq> <seed> [newRun c0]
//
// tests/test_binding_check.py runs it next to mdqt_run (the engine's own main loop) with the same
// inputs and requires every output file to be byte-identical.  Differences from the reference by
// design: srand48(seed) instead of srand48(time(NULL) + job) (:1219; a fixed seed for the
// comparison), the wavefunctions as std::complex<double>[12] per ion (the storage order of SpeedUp's
// 12x1 cx_mat: Armadillo is absent from the image), and the constants of the time loop read from the
// engine (the reference computes the same values in its globals, :79-85).
#include "mdqt.h"

#include <complex>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <cmath>
#include <vector>

// ---- SpeedUp's user inputs (:56-85; compile-time there, argv here) ----
static char saveDirectory[256] = "dataLaserCool/";
static double Ge = 0.1, tmax = 30, density = 2, sig0 = 4.0, Te = 19.0, fracOfSig = 0;
static double detuning = -1, detuningDP = 1, Om = 1, OmDP = 1;
static int N0 = 3500, newRun = 1, c0 = 0, sampleFreq = 40;
static unsigned seed = 12346;

// ---- SpeedUp's state (:111-160) ----
static std::vector<double> Rv, Vv, Fv, tPart;          // R,V,F[3][N0+1000], tPart[N0+1000]
static std::vector<std::complex<double>> wvFns;        // [N0+1000][12]: cx_mat wvFns[N0+1000] (12x1)
static size_t LD;                                      // N0 + 1000, the row stride of R, V, F
static double* R[3];
static double* V[3];
static int N;
static double L, t, Epot, Epot0;
static unsigned job;
static int plasmaToQuantumTimestepRatio;

// ---- the binding ----
static mdqt_ctx* g_mdqt = nullptr;

static void mdqt_or_die(int rc) {
    if (rc) { fprintf(stderr, "mdqt: %s\n", mdqt_last_error()); exit(1); }
}

static void mdqt_attach(unsigned jb) {                 // main() :1145, before saveDirectory is extended
    mdqt_params p;
    mdqt_default_params(&p);
    p.Ge = Ge; p.tmax = tmax; p.density = density; p.sig0 = sig0; p.Te = Te; p.fracOfSig = fracOfSig;
    p.detuning = detuning; p.detuningDP = detuningDP; p.Om = Om; p.OmDP = OmDP;
    p.N0 = N0; p.sampleFreq = sampleFreq; p.newRun = newRun; p.c0 = c0;
    p.seed = seed; p.job = jb;
    strncpy(p.saveDirectory, saveDirectory, sizeof(p.saveDirectory) - 1);
    mdqt_or_die(mdqt_create(&p, &g_mdqt));
    mdqt_or_die(mdqt_setup_directories(g_mdqt));       // the same tree as :1145-1160
    plasmaToQuantumTimestepRatio = (int)mdqt_get_const(g_mdqt, "plasmaToQuantumTimestepRatio");
}

static void push_state() {                             // host globals -> HBM
    std::vector<double> psi((size_t)N * 24);
    for (int i = 0; i < N; ++i)
        for (int k = 0; k < 12; ++k) {
            psi[24 * (size_t)i + 2 * k] = wvFns[12 * (size_t)i + k].real();
            psi[24 * (size_t)i + 2 * k + 1] = wvFns[12 * (size_t)i + k].imag();
        }
    mdqt_or_die(mdqt_set_state(g_mdqt, N, R[0], V[0], LD, psi.data(), tPart.data(), t));
}

static void push_counters() {                          // c0, the file counter and Epot0 of init()
    mdqt_or_die(mdqt_set_counters(g_mdqt, c0, 0u, Epot, Epot0));
}

static void pull_state() {                             // HBM -> host globals (after readConditions)
    N = mdqt_get_N(g_mdqt);
    std::vector<double> psi((size_t)N * 24);
    mdqt_or_die(mdqt_get_state(g_mdqt, R[0], V[0], nullptr, LD, psi.data(), tPart.data(), &t));
    for (int i = 0; i < N; ++i)
        for (int k = 0; k < 12; ++k)
            wvFns[12 * (size_t)i + k] = {psi[24 * (size_t)i + 2 * k], psi[24 * (size_t)i + 2 * k + 1]};
}

// ---- the hot-path functions (prototypes SpeedUp:176-185), bodies replaced ----
void forces(void) { mdqt_or_die(mdqt_forces(g_mdqt)); }                     // :192-236
void step(void) { mdqt_or_die(mdqt_step(g_mdqt)); }                         // :418-430
void qstep(void) { mdqt_or_die(mdqt_qstep(g_mdqt)); t = mdqt_get_time(g_mdqt); }   // :438-717
void Epotential(void) { mdqt_or_die(mdqt_epotential(g_mdqt, &Epot)); }      // :244-281
void output(void) { mdqt_or_die(mdqt_output(g_mdqt)); }                     // :917-1032
void writeConditions(int c) { mdqt_or_die(mdqt_write_conditions(g_mdqt, c)); }   // :725-784
void readConditions(int c) { mdqt_or_die(mdqt_read_conditions(g_mdqt, c)); pull_state(); }   // :785-916

// init(), SpeedUp:289-348: the reference's host sampling of N9L candidates from drand48, kept as is
// by the binding (restated), then the two appended lines
void init(void) {
    L = pow(N0 * 4. * M_PI / 3., 0.333333333);                                  // :297
    const double N9L = (unsigned)(9. * 9. * 9. * (L * L * L) * 3. / (4. * M_PI));   // :299
    N = 0;
    for (long i = 0; i < N9L; i++) {                                            // :303-335
        const double x = 9. * L * drand48() - 4. * L;
        const double y = 9. * L * drand48() - 4. * L;
        const double z = 9. * L * drand48() - 4. * L;
        if (x <= L && y <= L && z <= L && x > 0 && y > 0 && z > 0) {
            R[0][N] = x; R[1][N] = y; R[2][N] = z;
            V[0][N] = 0.; V[1][N] = 0.; V[2][N] = 0.;
            const double u1 = drand48(), u2 = drand48();
            const double sign = drand48() < 0.5 ? -1. : 1.;
            const double sign2 = drand48() < 0.5 ? -1. : 1.;
            std::complex<double>* w = &wvFns[12 * (size_t)N];
            for (int k = 0; k < 12; ++k) w[k] = 0.;
            w[0] = {sqrt(u1), 0.};
            w[1] = {sign2 * sqrt(1 - u1) * sqrt(u2), sign * sqrt(1 - u1) * sqrt(1 - u2)};
            tPart[N] = 0;
            N++;
        }
    }
    printf("%i\n", N);
    push_state();                                       // binding: the sampled state to HBM
    Epotential();                                       // :345-347
    Epot0 = Epot;
    c0 = -1;
    push_counters();                                    // binding: c0 and Epot0 to the engine
}

int main(int argc, char** argv) {
    if (argc < 7) {
        fprintf(stderr, "usage: %s <job> <saveDirectory/> <N0> <tmax> <sampleFreq> <seed> [newRun c0]\n", argv[0]);
        return 2;
    }
    job = (unsigned)atof(argv[1]);                     // :1145
    strncpy(saveDirectory, argv[2], sizeof(saveDirectory) - 1);
    N0 = atoi(argv[3]); tmax = atof(argv[4]); sampleFreq = atoi(argv[5]); seed = (unsigned)strtoul(argv[6], 0, 10);
    if (argc >= 9) { newRun = atoi(argv[7]); c0 = atoi(argv[8]); }
    LD = (size_t)N0 + 1000;
    Rv.assign(3 * LD, 0.); Vv.assign(3 * LD, 0.); Fv.assign(3 * LD, 0.); tPart.assign(LD, 0.);
    wvFns.assign(12 * LD, 0.);
    for (int k = 0; k < 3; ++k) { R[k] = Rv.data() + k * LD; V[k] = Vv.data() + k * LD; }
    mdqt_attach(job);                                   // the one line main() gains
    // (:1146-1215: the reference's directory tree and constant operators — the engine made both)
    srand48(seed);                                      // :1219 (time(NULL) + job in the reference)
    int timeStepCounter = plasmaToQuantumTimestepRatio; // :1235
    if (newRun == 1) init();                            // :1238-1246
    if (newRun == 0) readConditions(c0);
    while (t <= tmax + 0.0009) {                        // :1248
        if ((c0 + 1) % sampleFreq == 0 && timeStepCounter == 1) output();   // :1365-1368
        if (timeStepCounter == plasmaToQuantumTimestepRatio) {              // :1369-1375
            forces();
            c0++;
            timeStepCounter = 0;
        }
        step();                                         // :1376
        qstep();                                        // :1377
        timeStepCounter++;
    }
    writeConditions(c0);                                // :1381
    printf("binding_check: N=%d c0=%d t=%.9f dir=%s\n", N, c0, t, mdqt_save_directory(g_mdqt));
    mdqt_destroy(g_mdqt);
    return 0;
}
