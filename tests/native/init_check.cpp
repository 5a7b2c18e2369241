// Test driver for mdqtplasmasims_amd/csrc/mdqt_init_sample.hpp (tests/test_init_sample.py):
//   init_check <N0> <seed> <threads> <Nbound or 0>
// runs init()'s rejection sampling sequentially and with <threads> threads and exits 0 iff the
// kept ions (positions and wavefunction draws, bit for bit) and the final stream state agree.
#include "mdqt_init_sample.hpp"

#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>

int main(int argc, char** argv) {
    if (argc != 5) return 2;
    const long N0 = atol(argv[1]);
    const unsigned seed = (unsigned)atol(argv[2]);
    const int threads = atoi(argv[3]);
    long Nbound = atol(argv[4]);
    if (Nbound <= 0) Nbound = N0 + 1000 + (long)(20. * sqrt((double)N0 + 1.));
    const double L = pow(N0 * 4 * M_PI / 3, 0.333333333);                               // SpeedUp:297
    const double N9L = (unsigned)(9. * 9. * 9. * (L * L * L) * 3. / (4. * M_PI));      // :299
    uint64_t xs = 0, xp = 0;
    auto t0 = std::chrono::steady_clock::now();
    auto a = mdqt::init_sample(mdqt::srand48_state(seed), L, (long)N9L, Nbound, 1, &xs);
    auto t1 = std::chrono::steady_clock::now();
    auto b = mdqt::init_sample(mdqt::srand48_state(seed), L, (long)N9L, Nbound, threads, &xp);
    auto t2 = std::chrono::steady_clock::now();
    const bool same = a.size() == b.size() && xs == xp &&
                      (a.empty() || !memcmp(a.data(), b.data(), a.size() * sizeof(a[0])));
    printf("N=%zu %zu state %llx %llx same=%d seq %.3f s par %.3f s\n", a.size(), b.size(),
           (unsigned long long)xs, (unsigned long long)xp, (int)same,
           std::chrono::duration<double>(t1 - t0).count(), std::chrono::duration<double>(t2 - t1).count());
    return same ? 0 : 1;
}
