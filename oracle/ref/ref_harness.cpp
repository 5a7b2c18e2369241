// ORACLE — TEST INFRASTRUCTURE ONLY.
// C-ABI wrapper around the reference's own MD-only program, compiled UNMODIFIED from
// /root/reference/MonteCarloFollowedByMDAndTempAnisotropy.cpp (its main() is renamed by a
// -D flag so this file can call its functions).  It gives the tests the reference's own
// Yukawa force law / minimum image / cutoff (calculateAccelerations :387-448, calcAIJ
// :161-169), pair potential (calculatePotentialEnergyForParticles :207-244, calcUIJ :153-159)
// and position update + periodic wrap (stepPositions :453-467).
// Reference globals (N = 4096, kappa = 0.5, L = (4096*4pi/3)^(1/3)) are fixed by that file.
#include <cstring>
#include <omp.h>

extern double R[3][4096];
extern double V[3][4096];
extern double A[3][4096];
extern double U[4096];
extern double L;
extern double rCut;
void calculateAccelerations(int tS);
void calculatePotentialEnergyForParticles();
void stepPositions();
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
}
