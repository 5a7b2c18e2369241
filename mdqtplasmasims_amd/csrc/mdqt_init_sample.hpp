// init() sampling of laserCoolingPlusExpansionMDQTSpeedUp.cpp (:289-335) from one drand48 stream,
// sequential or in parallel with identical results (see mdqt_engine.cpp, mdqt_init).  Host only;
// header so that tests/native/init_check.cpp can compare the two paths at large N on the CPU.
#pragma once

#include <math.h>
#include <stdint.h>

#include <thread>
#include <vector>

namespace mdqt {

inline uint64_t srand48_state(uint32_t seed) { return (((uint64_t)seed) << 16) | 0x330Eull; }
inline double drand48_next(uint64_t* x) {
    *x = (0x5DEECE66Dull * (*x) + 0xBull) & 0xFFFFFFFFFFFFull;
    return (double)(*x) * 0x1p-48;             // = ldexp(x, -48): exact (x < 2^48)
}

struct Lcg48Jump {                       // 2^b steps of X' = A X + C (mod 2^48), b < 48
    uint64_t A[48], C[48];
    Lcg48Jump() {
        uint64_t a = 0x5DEECE66Dull, c = 0xBull;
        for (int b = 0; b < 48; ++b) {
            A[b] = a; C[b] = c;
            c = (a * c + c) & 0xFFFFFFFFFFFFull;
            a = (a * a) & 0xFFFFFFFFFFFFull;
        }
    }
    uint64_t jump(uint64_t x, uint64_t k) const {   // the state after k more draws
        for (int b = 0; k; ++b, k >>= 1)
            if (k & 1) x = (A[b] * x + C[b]) & 0xFFFFFFFFFFFFull;
        return x;
    }
};

struct InitIon { double x, y, z, w0, w2, w3; };

// the ion kept at draw index q: positions from u_q..u_q+2, wavefunction from u_q+3..u_q+6
inline InitIon init_ion(uint64_t state_before_q, double L) {
    uint64_t x = state_before_q;
    InitIon r;
    r.x = 9. * L * drand48_next(&x) - 4. * L;
    r.y = 9. * L * drand48_next(&x) - 4. * L;
    r.z = 9. * L * drand48_next(&x) - 4. * L;
    const double rand1 = drand48_next(&x);                                             // :317-328
    const double rand2 = drand48_next(&x);
    const double rand3 = drand48_next(&x);
    double sign = 1;
    if (rand3 < 0.5) sign = -1;
    const double rand4 = drand48_next(&x);
    double sign2 = 1;
    if (rand4 < 0.5) sign2 = -1;
    r.w0 = sqrt(rand1);                                                                // :329-332
    r.w2 = sign2 * sqrt(1 - rand1) * sqrt(rand2);
    r.w3 = sign * sqrt(1 - rand1) * sqrt(1 - rand2);
    return r;
}

inline bool init_ok(double u, double L) {
    const double x = 9. * L * u - 4. * L;
    return x <= L && x > 0;                                                            // :308
}

// returns the kept ions in stream order and the stream state after the last candidate
inline std::vector<InitIon> init_sample(uint64_t seed_state, double L, long N9L, long Nbound, int threads,
                                 uint64_t* final_state) {
    std::vector<InitIon> out;
    out.reserve((size_t)Nbound);
    if (threads <= 1 || N9L < 3 * 4096) {                                            // :303-335
        uint64_t x = seed_state;
        for (long i = 0; i < N9L; i++) {
            const uint64_t before = x;
            const double u0 = drand48_next(&x), u1 = drand48_next(&x), u2 = drand48_next(&x);
            const bool ok = init_ok(u0, L) && init_ok(u1, L) && init_ok(u2, L);
            if (ok) {
                out.push_back(init_ion(before, L));
                for (int k = 0; k < 4; ++k) drand48_next(&x);
            }
        }
        *final_state = x;
        return out;
    }
    static const Lcg48Jump J;
    // (1) scan draw indices [0, P) for the starts of keepable triples
    const uint64_t P = 3ull * (uint64_t)N9L + 4ull * (uint64_t)Nbound + 8;
    std::vector<std::vector<uint64_t>> found(threads);
    {
        std::vector<std::thread> pool;
        for (int t = 0; t < threads; ++t)
            pool.emplace_back([&found, t, P, threads, seed_state, L] {
                const uint64_t a = P * t / threads, b = P * (t + 1) / threads;
                uint64_t x = J.jump(seed_state, a);
                std::vector<uint64_t> mine;
                // m: ok flags of the last three draws (bit 0 = newest); after the draw of
                // u_{p+2}, m == 7 iff the candidate starting at p is kept
                unsigned m = (unsigned)init_ok(drand48_next(&x), L) << 1 | (unsigned)init_ok(drand48_next(&x), L);
                for (uint64_t p = a; p < b; ++p) {
                    m = ((m << 1) | (unsigned)init_ok(drand48_next(&x), L)) & 7u;
                    if (__builtin_expect(m == 7u, 0)) mine.push_back(p);
                }
                found[t] = std::move(mine);
            });
        for (auto& th : pool) th.join();
    }
    std::vector<uint64_t> cls[3];
    for (auto& f : found)
        for (uint64_t p : f) cls[p % 3].push_back(p);
    found.clear();
    // (2) walk the candidates
    std::vector<uint64_t> kept;
    kept.reserve((size_t)Nbound);
    size_t ptr[3] = {0, 0, 0};
    uint64_t p = 0;
    uint64_t cand = 0;
    const uint64_t ncand = (uint64_t)N9L;
    bool covered = true;
    while (cand < ncand) {
        const int c = (int)(p % 3);
        auto& v = cls[c];
        size_t& i = ptr[c];
        while (i < v.size() && v[i] < p) ++i;
        if (i == v.size()) {
            // no listed start in this class at or after p: the walk is covered up to P only
            const uint64_t last = p + 3 * (ncand - cand - 1);    // start of the final candidate
            if (last + 2 < P) { p += 3 * (ncand - cand); cand = ncand; break; }
            covered = false;
            break;
        }
        const uint64_t q = v[i];
        const uint64_t skip = (q - p) / 3;                         // rejected candidates before q
        if (cand + skip >= ncand) { p += 3 * (ncand - cand); cand = ncand; break; }
        if (q + 2 >= P) { covered = false; break; }
        kept.push_back(q);
        cand += skip + 1;
        p = q + 7;
    }
    // (3) the kept ions' draws, in parallel by jump-ahead
    out.resize(kept.size());
    {
        std::vector<std::thread> pool;
        for (int t = 0; t < threads; ++t)
            pool.emplace_back([&, t] {
                const size_t a = kept.size() * t / threads, b = kept.size() * (t + 1) / threads;
                for (size_t k = a; k < b; ++k) out[k] = init_ion(J.jump(seed_state, kept[k]), L);
            });
        for (auto& th : pool) th.join();
    }
    uint64_t x = J.jump(seed_state, p);
    if (!covered) {                                             // finish sequentially from p
        for (; cand < ncand; ++cand) {
            const uint64_t before = x;
            const double u0 = drand48_next(&x), u1 = drand48_next(&x), u2 = drand48_next(&x);
            const bool ok = init_ok(u0, L) && init_ok(u1, L) && init_ok(u2, L);
            if (ok) {
                out.push_back(init_ion(before, L));
                for (int k = 0; k < 4; ++k) drand48_next(&x);
            }
        }
    }
    *final_state = x;
    return out;
}


}  // namespace mdqt
