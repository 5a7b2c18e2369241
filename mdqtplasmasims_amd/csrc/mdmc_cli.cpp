// mdmc — drop-in command line for MonteCarloFollowedByMDAndTempAnisotropy.cpp and, with
// --qt_model=1|2|3, for MonteCarloFollowedByQTTagging408Linear.cpp / 408Quad.cpp / 422Linear.cpp.
//
//   reference:  ./a.out <job>                      (MCMD:1035; parameters are globals :62-107)
//   this:       mdmc <job> [--qt_model=m] [--Name=value ...]   (same parameter names and defaults;
//               --qt_model selects the tagging program and its defaults, QTT:75-121)
//
// Runs main()'s stages (MCMD:1030-1167) on the GPU through include/mdmc.h and writes the same
// directory tree and files (pairPairCorrStepNum%d.dat, temperature.dat, VAF.dat, ...).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mdmc.h"
#include "mdqt.h"

static void usage(void) {
    fprintf(stderr,
            "usage: mdmc <job> [--N=4096] [--kappa=0.5] [--Gamma=3] [--n=0.4] [--collisionFreq=0.25]\n"
            "                  [--monteCarloSteps=200000] [--maxRStep=0.3] [--pairPairStep=0.05]\n"
            "                  [--timeStep=0.005] [--numPreRecordMDSteps=200] [--numVelAutoCorrsSteps=2500]\n"
            "                  [--numInstantaneousAnisotropySteps=2500] [--numReestablishEquilSteps=500]\n"
            "                  [--tempPercentDiff=0.15] [--applyForceAlongOneAxisOnly=0] [--beta=26000]\n"
            "                  [--anisotropyEstablishmentTime=10] [--anisotropyFromForcesRelaxSteps=2000]\n"
            "                  [--saveDirectory=data/] [--seed=<mt19937 seed; default time(NULL)+job>]\n"
            "                  [--device=-1] [--force_kernel=1] [--quiet=0]\n"
            "                  [--qt_model=0|1|2|3] [--tpumpreal=2e-7] [--detuning=-2.5] [--Om=0.7]\n");
}

int main(int argc, char** argv) {
    if (argc < 2) { usage(); return 2; }
    mdmc_params p;
    mdmc_default_params(&p);
    for (int i = 2; i < argc; ++i)                          // the tagging program's defaults first
        if (!strncmp(argv[i], "--qt_model=", 11) && atoi(argv[i] + 11) != 0) {
            if (mdmc_default_params_qt(&p, atoi(argv[i] + 11)) != 0) {
                fprintf(stderr, "mdmc: %s\n", mdqt_last_error());
                return 2;
            }
        }
    const double job = atof(argv[1]);                       // MCMD:1035
    p.job = (uint32_t)job;
    int seed_given = 0, quiet = 0;
    for (int i = 2; i < argc; ++i) {
        const char* a = argv[i];
        if (strncmp(a, "--", 2) != 0 || !strchr(a, '=')) { usage(); return 2; }
        char key[64];
        const char* eq = strchr(a, '=');
        size_t kl = (size_t)(eq - a - 2);
        if (kl >= sizeof key) { usage(); return 2; }
        memcpy(key, a + 2, kl);
        key[kl] = 0;
        const char* v = eq + 1;
#define DPAR(name) if (!strcmp(key, #name)) { p.name = atof(v); continue; }
#define IPAR(name) if (!strcmp(key, #name)) { p.name = atoi(v); continue; }
        DPAR(kappa) DPAR(Gamma) DPAR(n) DPAR(collisionFreq) DPAR(maxRStep) DPAR(pairPairStep) DPAR(timeStep)
        DPAR(tempPercentDiff) DPAR(beta) DPAR(tpumpreal) DPAR(detuning) DPAR(Om)
        IPAR(N) IPAR(monteCarloSteps) IPAR(numPreRecordMDSteps) IPAR(numVelAutoCorrsSteps)
        IPAR(numInstantaneousAnisotropySteps) IPAR(numReestablishEquilSteps) IPAR(applyForceAlongOneAxisOnly)
        IPAR(anisotropyEstablishmentTime) IPAR(anisotropyFromForcesRelaxSteps) IPAR(device) IPAR(force_kernel)
        IPAR(qt_model)
#undef DPAR
#undef IPAR
        if (!strcmp(key, "quiet")) { quiet = atoi(v); continue; }
        if (!strcmp(key, "seed")) { p.seed = (uint32_t)strtoul(v, NULL, 10); seed_given = 1; continue; }
        if (!strcmp(key, "saveDirectory")) {
            strncpy(p.saveDirectory, v, sizeof(p.saveDirectory) - 1);
            continue;
        }
        fprintf(stderr, "mdmc: unknown parameter %s\n", key);
        return 2;
    }
    if (!seed_given) p.seed = (uint32_t)(time(NULL) + job);   // the reference: std::random_device (:52)
    mdmc_ctx* c = NULL;
    if (mdmc_create(&p, &c) != 0) {
        fprintf(stderr, "mdmc: %s\n", mdqt_last_error());
        return 1;
    }
    const int rc = mdmc_run(c, !quiet);
    if (rc != 0) fprintf(stderr, "mdmc: %s\n", mdqt_last_error());
    mdmc_destroy(c);
    return rc ? 1 : 0;
}
