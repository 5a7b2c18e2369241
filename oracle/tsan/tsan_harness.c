/* ORACLE — TEST INFRASTRUCTURE ONLY.  ThreadSanitizer check of the oracle's OpenMP loops
 * (the CPU restatement must be race-free, unlike the reference's forces() scatter,
 * SpeedUp:228-230, and its shared drand48 in qstep(), SpeedUp:486).
 *   tsan_harness oracle    run forces() + qsteps + observables of the restatement on 4 threads
 *   tsan_harness control   a deliberately racy loop (the reference's Newton-3 scatter pattern):
 *                          the positive control that shows the sanitizer sees OpenMP races
 * Built by oracle/tsan/Makefile with clang -fsanitize=thread and LLVM's libomp; run with
 * OMP_TOOL_LIBRARIES=libarcher.so so that TSan knows OpenMP's synchronisation. */
#include <stdio.h>
#include <string.h>
#include "../mdqt_oracle.h"

static int run_oracle(void) {
    orc_params p;
    orc_default_params(&p);
    p.N0 = 300; p.rng_mode = 1; p.nthreads = 4; p.seed = 7; p.job = 1;
    orc_sim* s = orc_create(&p);
    if (!s || orc_init(s)) return 1;
    orc_md_steps(s, 2);                          /* forces_rows + substeps (OpenMP over ions) */
    double o7[7];
    orc_observables(s, o7, NULL, NULL);
    printf("oracle N=%d t=%g Ekin_x=%g\n", orc_get_N(s), orc_get_time(s), o7[1]);
    orc_destroy(s);
    return 0;
}

static int run_control(void) {
    enum { N = 512 };
    static double F[N];
    memset(F, 0, sizeof F);
#pragma omp parallel for num_threads(4) schedule(static, 1)
    for (int i = 0; i < N - 1; i++)
        for (int j = i + 1; j < N; j++) {        /* F[i] += f; F[j] -= f from different threads */
            F[i] += 1e-3;
            F[j] -= 1e-3;
        }
    double t = 0;
    for (int i = 0; i < N; i++) t += F[i];
    printf("control sum=%g\n", t);
    return 0;
}

int main(int argc, char** argv) {
    if (argc > 1 && !strcmp(argv[1], "control")) return run_control();
    return run_oracle();
}
