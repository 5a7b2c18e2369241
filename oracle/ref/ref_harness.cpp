// ORACLE — TEST INFRASTRUCTURE ONLY.
// C-ABI wrapper around the reference's own MD-only program, compiled UNMODIFIED from
// /root/reference/MonteCarloFollowedByMDAndTempAnisotropy.cpp (its main() is renamed by a
// -D flag so this file can call its functions).  It gives the tests the reference's own
// Yukawa force law / minimum image / cutoff (calculateAccelerations :387-448, calcAIJ
// :161-169), pair potential (calculatePotentialEnergyForParticles :207-244, calcUIJ :153-159),
// position update + periodic wrap (stepPositions :453-467), and — with its global mt19937
// reseeded (the reference seeds it from std::random_device, :52-53) — its init (:173-203),
// Metropolis MC (:315-382), velocity-Verlet MD with collisions (:469-511), g(r) (:584-652),
// velocity autocorrelations (:655-807), tagging (:810-921, :923-1028) and temperatures.
// Reference globals (N = 4096, kappa = 0.5, Gamma = 3, L = (4096*4pi/3)^(1/3)) are fixed by that file.
#include <cstdio>
#include <cstring>
#include <omp.h>
#include <random>

extern double R[3][4096];
extern double V[3][4096];
extern double A[3][4096];
extern double U[4096];
extern double L;
extern double rCut;
extern double collisionFreq;
extern int addLaserForce;
extern char saveDirectory[256];
extern std::mt19937 rng;
extern std::uniform_real_distribution<double> uni;
extern std::normal_distribution<double> velocityDistribution;
extern double vStore[3][4096][2500];
extern double VAF[2500];
extern double longViscAutoCorr[2500];
extern double vCubeAutoCorr[2500];
extern double vFourthAutoCorr[2500];
extern bool taggedOne[4096], taggedTwo[4096], taggedThree[4096], taggedFour[4096];
void init();
void MonteCarloStep();
void calculateAccelerations(int tS);
void calculatePotentialEnergyForParticles();
void stepPositions();
void MDStep(int tS);
void recordPairPairCorr(int stepNum);
void recordVAF(void);
void recordLongViscAutoCorr(void);
void recordVCubeAutoCorr(void);
void recordVFourthAutoCorr(void);
void recordTemperature(void);
void tagParticles();
void recordTaggedParticleMoments(int step);
void recordTempForEachAxis(char fileName[256], int step);
double calcUIJ(double totalDist);
double calcAIJ(double totalDist);

extern "C" {
int mdref_N() { return 4096; }
double mdref_L() { return L; }
double mdref_rcut() { return rCut; }
double mdref_kappa() { return 0.5; }
double mdref_uij(double r) { return calcUIJ(r); }
double mdref_aij(double r) { return calcAIJ(r); }
// Rin, Aout: [3][4096]
void mdref_accelerations(const double* Rin, double* Aout) {
    std::memcpy(R, Rin, sizeof(R));
    omp_set_num_threads(1);  // the reference loop races on A[j] under >1 thread
    calculateAccelerations(0);
    std::memcpy(Aout, A, sizeof(A));
}
// per-particle potential energy U[i] = sum_{j != i} u(r_ij)
void mdref_particle_potentials(const double* Rin, double* Uout) {
    std::memcpy(R, Rin, sizeof(R));
    calculatePotentialEnergyForParticles();
    std::memcpy(Uout, U, sizeof(U));
}
// R <- R + dt V + dt^2/2 A (dt = 0.005) with the periodic re-insertion
void mdref_step_positions(double* Rio, const double* Vin, const double* Ain) {
    std::memcpy(R, Rio, sizeof(R));
    std::memcpy(V, Vin, sizeof(V));
    std::memcpy(A, Ain, sizeof(A));
    stepPositions();
    std::memcpy(Rio, R, sizeof(R));
}

// ---- seeded program stages (the reference's own code; only the seed is ours) ----
// the program's state right after its static initialisation, with seed s: zeroed globals
// (R, V, A, U, :110-123 — the first MDStep reads A as oldA), mt19937 seeded, one uniform drawn by
// `auto random_double = uni(rng);` (:52-55)
void mdref_seed(unsigned s) {
    std::memset(R, 0, sizeof(R));
    std::memset(V, 0, sizeof(V));
    std::memset(A, 0, sizeof(A));
    std::memset(U, 0, sizeof(U));
    rng.seed(s);
    uni.reset();
    velocityDistribution.reset();
    (void)uni(rng);
}
void mdref_set_collision_freq(double f) { collisionFreq = f; }
void mdref_set_laser_force(int on) { addLaserForce = on; }
void mdref_set_save_directory(const char* d) {
    std::strncpy(saveDirectory, d, sizeof(saveDirectory) - 1);
    saveDirectory[sizeof(saveDirectory) - 1] = 0;
}
void mdref_get(double* Ro, double* Vo, double* Ao, double* Uo) {
    if (Ro) std::memcpy(Ro, R, sizeof(R));
    if (Vo) std::memcpy(Vo, V, sizeof(V));
    if (Ao) std::memcpy(Ao, A, sizeof(A));
    if (Uo) std::memcpy(Uo, U, sizeof(U));
}
void mdref_set(const double* Ri, const double* Vi, const double* Ai, const double* Ui) {
    if (Ri) std::memcpy(R, Ri, sizeof(R));
    if (Vi) std::memcpy(V, Vi, sizeof(V));
    if (Ai) std::memcpy(A, Ai, sizeof(A));
    if (Ui) std::memcpy(U, Ui, sizeof(U));
}
void mdref_init() { init(); calculatePotentialEnergyForParticles(); }   // main() steps 1-2 (:1062-1065)
void mdref_monte_carlo(int n) { for (int k = 0; k < n; ++k) MonteCarloStep(); }
void mdref_md_steps(int n) {
    omp_set_num_threads(1);
    for (int k = 0; k < n; ++k) MDStep(k);
}
void mdref_pair_corr(int step) { recordPairPairCorr(step); }          // writes pairPairCorrStepNum<k>.dat
// vin: [3][4096][T] (T <= 2500, the rest zero); out: VAF, longVisc, vCube, vFourth [4][2500]
void mdref_autocorrelations(const double* vin, int T, double* out) {
    std::memset(vStore, 0, sizeof(vStore));
    for (int c = 0; c < 3; ++c)
        for (int i = 0; i < 4096; ++i)
            for (int t = 0; t < T; ++t) vStore[c][i][t] = vin[((size_t)c * 4096 + i) * T + t];
    recordVAF();
    recordLongViscAutoCorr();
    recordVCubeAutoCorr();
    recordVFourthAutoCorr();
    std::memcpy(out, VAF, sizeof(VAF));
    std::memcpy(out + 2500, longViscAutoCorr, sizeof(VAF));
    std::memcpy(out + 5000, vCubeAutoCorr, sizeof(VAF));
    std::memcpy(out + 7500, vFourthAutoCorr, sizeof(VAF));
}
void mdref_record_temperature() { recordTemperature(); }              // appends temperature.dat
void mdref_record_temp_axes(int step) {                               // appends tempAxes.dat
    char f[256];
    std::snprintf(f, sizeof f, "%stempAxes.dat", saveDirectory);
    recordTempForEachAxis(f, step);
}
void mdref_tag_particles(int* tags4) {                                  // [4][4096]
    tagParticles();
    for (int i = 0; i < 4096; ++i) {
        tags4[i] = taggedOne[i]; tags4[4096 + i] = taggedTwo[i];
        tags4[8192 + i] = taggedThree[i]; tags4[12288 + i] = taggedFour[i];
    }
}
void mdref_tagged_moments(int step) { recordTaggedParticleMoments(step); }   // appends taggedV*Moments.dat
}
