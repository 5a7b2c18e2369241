/*
 * mdmc.h — C ABI of the MI355X engine for the reference's Monte-Carlo + MD analytics program
 *   MonteCarloFollowedByMDAndTempAnisotropy.cpp        ("MCMD" below, tlangin/MDQTPlasmaSims)
 * (SURVEY §8(f)4).  The reference's seam is a set of functions over globals (MCMD:130-147)
 * driven by main() (MCMD:1030-1167); every entry point below names the function it replaces.
 *
 * RNG: the reference's own std::mt19937 (seeded from std::random_device, MCMD:52-53; here from
 * `seed`) with std::uniform_real_distribution<double>(0,1) and std::normal_distribution
 * (MCMD:54, :87), consumed in the reference's order: the Metropolis draws inside the device
 * MC kernel (mt19937 + libstdc++ generate_canonical<double, 53> on the GPU, the state handed
 * over from and back to the host engine), the Maxwell-Boltzmann velocities, collision rolls and
 * tag rolls on the host.  With the same seed the trajectory follows the reference program's
 * stream: the Metropolis energy change is summed in a fixed tree order (and, with force_kernel 1,
 * from reciprocal-form pair energies with a polynomial exp) where the reference sums
 * sequentially with libm exp (MCMD:341-357), so an accept decision whose dice lies within a few
 * ulp of exp(-dE Gamma / 2) can go the other way — the stream then shifts and the runs part
 * statistically.  The parity tests pin 3,000 MC steps bit for bit against the reference build;
 * longer horizons are statistical parity, not a bitwise guarantee.
 *
 * Conventions as include/mdqt.h: opaque context, int status (0 ok, <0 error; message in
 * mdqt_last_error()), caller-owned host buffers, R/V/A as [3][N] row-major like the reference's
 * `double R[3][N]` (MCMD:110-112), device state resident between calls.
 *
 * The same engine runs the QT spin-tagging variants of the program ("QTT":
 * MonteCarloFollowedByQTTagging408Linear.cpp / 408Quad.cpp / 422Linear.cpp; qt_model 1 / 2 / 3):
 * the same MC anneal and collisional MD, then a pump period of QT steps (the optical-pumping
 * qstep of include/mdqt.h's qt_model, QTT:555, driven by this system's velocities) between MD
 * steps, QT tagging (QTT:1022) and collisionless MD recording the tagged ions' moments and
 * velocity distribution (QTT:1069-1138) and the autocorrelations.  Wavefunctions start as the
 * reference's random S superpositions from its drand48 stream (default seed, QTT:224-239); the
 * QT jump draws use the Philox stream of include/mdqt.h (keyed by seed, job, ion, qstep index)
 * instead of the reference's shared drand48.
 */
#ifndef MDMC_H
#define MDMC_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

/* The reference's compile-time inputs (MCMD:62-107), same names, same defaults. */
typedef struct mdmc_params {
    int N;                        /* :66  particles; a perfect cube (cubic-lattice init :182-201) */
    double kappa;                 /* :67  screening parameter                                    */
    double Gamma;                 /* :68  coupling (inverse normalised temperature)              */
    double n;                     /* :69  density (1e14 m^-3): laser-force units (:491-496)      */
    double collisionFreq;         /* :75  collision rate of the collisional MD stages           */
    int monteCarloSteps;          /* :80                                                         */
    double maxRStep;              /* :81  largest MC displacement                                */
    double pairPairStep;          /* :82  g(r) bin width (units of a)                            */
    double timeStep;              /* :88                                                         */
    int numPreRecordMDSteps;      /* :89                                                         */
    int numVelAutoCorrsSteps;     /* :90                                                         */
    int numInstantaneousAnisotropySteps; /* :96                                                  */
    int numReestablishEquilSteps; /* :97                                                         */
    double tempPercentDiff;       /* :98                                                         */
    int applyForceAlongOneAxisOnly; /* :103                                                      */
    double beta;                  /* :104 heating / cooling rate (s^-1)                          */
    int anisotropyEstablishmentTime; /* :105 (us)                                                */
    int anisotropyFromForcesRelaxSteps; /* :107                                                  */
    /* ---- extensions ---- */
    uint32_t seed;                /* mt19937 seed (reference: std::random_device, :52-53)       */
    uint32_t job;                 /* argv[1] (:1035)                                             */
    int device;                   /* HIP device ordinal (-1 = current)                           */
    int force_kernel;             /* 1 (default): reciprocal pair forms (MD forces, MC energies;
                                   * a few ulp per pair), 0: the reference's operations          */
    /* ---- QT tagging variants (QTT:84-121) ---- */
    int qt_model;                 /* 0: MCMD (no QT); 1: 408 linear, 2: 408 quad, 3: 422 linear    */
    double tpumpreal;             /* QTT:85 pump time (s)                                          */
    double detuning;              /* QTT:86 pump detuning (units of gamma)                         */
    double Om;                    /* QTT:87 Rabi frequency (units of gamma)                        */
    char saveDirectory[256];      /* :62 */
} mdmc_params;

typedef struct mdmc_ctx mdmc_ctx;

void        mdmc_default_params(mdmc_params* p);              /* MCMD:62-107 defaults         */
/* the QT tagging program's defaults (QTT:75-121: n = 2, 100000 MC steps, 1500 recorded steps,
 * the model's pump time, detuning, Rabi frequency and save directory); model 1..3 */
int         mdmc_default_params_qt(mdmc_params* p, int model);
int         mdmc_create(const mdmc_params* p, mdmc_ctx** out); /* + rng (:52-55), L, rCut (:73-74) */
void        mdmc_destroy(mdmc_ctx* c);
/* "N", "L", "rCut", "nbins", "collisionFreq"; QT: "plasmaToQuantumTimestepRatio",
 * "quantumTimestep", "gamToEinsteinFreq", "plasVelToQuantVel", "decayRatio", "pumpMDTimeSteps" */
double      mdmc_get_const(const mdmc_ctx* c, const char* name);

/* ---- the program's functions ---- */
int mdmc_init(mdmc_ctx* c);                 /* init() :173-203 + calculatePotentialEnergyForParticles() :207-245 */
int mdmc_monte_carlo(mdmc_ctx* c, int nsteps, long long* accepted); /* MonteCarloStep() x n, :315-382 */
int mdmc_md_steps(mdmc_ctx* c, int nsteps); /* MDStep() x n, :504-511 (stepPositions, calculateAccelerations,
                                             * stepVelocities with collisions and laser force :452-502) */
int mdmc_set_collision_freq(mdmc_ctx* c, double f); /* collisionFreq = f (main :1093, :1125, :1139) */
int mdmc_set_laser_force(mdmc_ctx* c, int on);      /* addLaserForce (main :1138, :1155)              */
/* recordPairPairCorr :584-652: g[nbins], nbins = (int)((L/2) / pairPairStep) (the file's rows) */
int mdmc_pair_corr(mdmc_ctx* c, double* g, int cap, int* nbins);
int mdmc_record_velocities(mdmc_ctx* c, int k);     /* recordVelsForAutocorrelations :513-523   */
/* recordVAF / recordLongViscAutoCorr / recordVCubeAutoCorr / recordVFourthAutoCorr :655-807 over
 * the stored velocities: out [4][numVelAutoCorrsSteps] */
int mdmc_autocorrelations(mdmc_ctx* c, double* out);
int mdmc_set_velocity_store(mdmc_ctx* c, const double* vs); /* [3][N][numVelAutoCorrsSteps] (tests) */
/* out4 = <v^2> over all components (recordTemperature :525-546), <vx^2>, <vy^2>, <vz^2> (:560-581) */
int mdmc_temperatures(mdmc_ctx* c, double out4[4]);
int mdmc_anisotropize(mdmc_ctx* c);                 /* anisotropizeVelocities :548-558          */
int mdmc_tag_particles(mdmc_ctx* c, int* tags4);    /* tagParticles :810-921; tags4 [4][N] or NULL */
/* recordTaggedParticleMoments :923-1028: out16 = (first, second - 1/Gamma, third,
 * fourth - 3/Gamma^2) for taggedOne .. taggedFour */
int mdmc_tagged_moments(mdmc_ctx* c, double out16[16]);
int mdmc_get_state(mdmc_ctx* c, double* R, double* V, double* A, double* U);    /* NULL = skip */
int mdmc_set_state(mdmc_ctx* c, const double* R, const double* V, const double* A, const double* U);
int mdmc_setup_directories(mdmc_ctx* c);            /* main() :1037-1058                        */
const char* mdmc_save_directory(const mdmc_ctx* c);
int mdmc_run(mdmc_ctx* c, int verbose);             /* main() :1030-1167 (QTT: :1140-1254): every stage and file */

/* ---- QT tagging variants (qt_model 1..3) ---- */
int mdmc_qsteps(mdmc_ctx* c, int n);                /* qstep() x n (QTT:555-756), velocities read from the MD state */
/* tagParticles (QTT:1022-1067): tags [N] 0/1 (or NULL), *n_up = number tagged (or NULL) */
int mdmc_tag_qt(mdmc_ctx* c, int* tags, int* n_up);
/* recordTaggedParticleMoments (QTT:1069-1138): out4 = first .. fourth moment of vx over the tagged
 * ions; dist (or NULL) = [3][4001] normalised velocity distributions of the tagged ions on the
 * bins (j - 2000) * 0.0025 (the reference writes the x row to vel_distX_timestep%06d.dat) */
int mdmc_tagged_moments_qt(mdmc_ctx* c, double out4[4], double* dist);
int mdmc_get_psi(mdmc_ctx* c, double* psi);         /* [N][12][2] (re, im; states past the model's zero) */
int mdmc_set_psi(mdmc_ctx* c, const double* psi);

#ifdef __cplusplus
}
#endif
#endif /* MDMC_H */
