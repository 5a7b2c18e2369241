// mdqt — drop-in command line for laserCoolingPlusExpansionMDQTSpeedUp.cpp.
//
//   reference:  ./a.out <job>                      (SpeedUp:1145, parameters are #defines :56-85)
//   this:       mdqt <job> [--Name=value ...]      (same parameter names and defaults)
//
// Writes the same directory tree (SpeedUp:1143-1160) and the same files
// (energies.dat, vel_dist{X,Y,Z}_time%06d.dat, statePopulationsVsVTime%06d.dat,
// ions_/conditions_/VZERO_/wvFns_timestep%06d.dat) through the C ABI of include/mdqt.h.
//
//   --pump_program=1|2|3 runs instead the main() of randomFrozenStartTag408Linear.cpp /
//   408Quad.cpp / 422Linear.cpp (their defaults, :52-80; mdqt_run_pump): the PumpTime...
//   directory, spinUpIons_*, taggedMoments.dat, tagged vel_distX_*, VAF.dat, the conditions.
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

#include "mdqt.h"

static void usage(void) {
    fprintf(stderr,
            "usage: mdqt <job> [--Ge=0.1] [--tmax=30] [--density=2] [--sig0=4] [--Te=19]\n"
            "                  [--fracOfSig=0] [--detuning=-1] [--detuningDP=1] [--Om=1] [--OmDP=1]\n"
            "                  [--N0=3500] [--newRun=1] [--c0=0] [--sampleFreq=40]\n"
            "                  [--reNormalizewvFns=0] [--saveDirectory=dataLaserCool/]\n"
            "                  [--seed=<srand48 seed; default time(NULL)+job as SpeedUp:1219>]\n"
            "                  [--qt=1] [--device=-1]\n"
            "       mdqt <job> --pump_program=1|2|3 [--tpumpreal=2e-7] [--tstartV0=15] [... as above]\n");
}

int main(int argc, char** argv) {
    if (argc < 2) { usage(); return 2; }
    mdqt_params p;
    mdqt_default_params(&p);
    int pump = 0;                                           // the pumping programs' defaults first
    for (int i = 2; i < argc; ++i)
        if (!strncmp(argv[i], "--pump_program=", 15)) pump = atoi(argv[i] + 15);
    if (pump < 0 || pump > 3) { usage(); return 2; }
    if (pump) mdqt_default_params_pump(&p, pump);
    const double job = atof(argv[1]);                       // SpeedUp:1145
    p.job = (uint32_t)job;
    int seed_given = 0;
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
        DPAR(Ge) DPAR(tmax) DPAR(density) DPAR(sig0) DPAR(Te) DPAR(fracOfSig) DPAR(detuning)
        DPAR(detuningDP) DPAR(Om) DPAR(OmDP) DPAR(tpumpreal) DPAR(tstartV0)
        IPAR(N0) IPAR(newRun) IPAR(c0) IPAR(sampleFreq) IPAR(reNormalizewvFns) IPAR(device) IPAR(qt_model)
#undef DPAR
#undef IPAR
        if (!strcmp(key, "qt")) { p.qt_enabled = atoi(v); continue; }
        if (!strcmp(key, "pump_program")) continue;         // applied above
        if (!strcmp(key, "seed")) { p.seed = (uint32_t)strtoul(v, NULL, 10); seed_given = 1; continue; }
        if (!strcmp(key, "saveDirectory")) {
            strncpy(p.saveDirectory, v, sizeof(p.saveDirectory) - 1);
            continue;
        }
        fprintf(stderr, "mdqt: unknown parameter %s\n", key);
        return 2;
    }
    if (!seed_given) p.seed = (uint32_t)(time(NULL) + job);   // SpeedUp:1219
    mdqt_ctx* c = NULL;
    if (mdqt_create(&p, &c)) {
        fprintf(stderr, "mdqt: %s\n", mdqt_last_error());
        return 1;
    }
    int rc = pump ? mdqt_run_pump(c) : mdqt_run(c);
    if (rc) fprintf(stderr, "mdqt: %s\n", mdqt_last_error());
    else printf("%i\n", mdqt_get_N(c));
    mdqt_destroy(c);
    return rc ? 1 : 0;
}
