// oracle/stdgen.hpp — TEST INFRASTRUCTURE ONLY (parity checker).
//
// Restatement of random-1.1 `System.Random.StdGen` (L'Ecuyer combined MLCG),
// the generator behind the reference's `Delays` draws
// (examples/token-ring/Main.hs:9,60,77: `mkStdGen 0`, `getRandomTR networkDelay`).
// random-1.1 is an un-vendored dependency (lts-7.9, time-warp.cabal:69): its
// source is not in /root/reference; this follows the published algorithm
// (SURVEY.md Appendix C).  PARITY UNPINNED: no reference test pins a draw.
#pragma once
#include <cstdint>

struct StdGen {
    int32_t s1, s2;
};

// mkStdGen s = mkStdGen32 (fromIntegral s)
inline StdGen mk_stdgen(int64_t seed) {
    int32_t s32 = (int32_t)(uint32_t)(uint64_t)seed;   // fromIntegral :: Int -> Int32
    int32_t s = s32 & 0x7fffffff;                       // .&. maxBound
    int32_t q = s / 2147483562, s1 = s % 2147483562;    // divMod (s >= 0)
    int32_t s2 = q % 2147483398;
    return StdGen{s1 + 1, s2 + 1};
}

// stdNext: returns z in [1, 2147483562]
inline int32_t stdgen_next(StdGen& g) {
    int32_t k = g.s1 / 53668;
    int32_t s1 = 40014 * (g.s1 - k * 53668) - k * 12211;
    if (s1 < 0) s1 += 2147483563;
    int32_t k2 = g.s2 / 52774;
    int32_t s2 = 40692 * (g.s2 - k2 * 52774) - k2 * 3791;
    if (s2 < 0) s2 += 2147483399;
    g.s1 = s1;
    g.s2 = s2;
    int32_t z = s1 - s2;
    if (z < 1) z += 2147483562;
    return z;
}

// randomR (lo, hi) via randomIvalInteger: accumulate base-b digits (b = 2147483562,
// genRange = (1, 2147483562)) until the magnitude reaches k*1000, then lo + v mod k.
inline int64_t stdgen_range(StdGen& g, int64_t lo, int64_t hi) {
    if (lo > hi) { int64_t t = lo; lo = hi; hi = t; }
    const __int128 b = 2147483562;
    const __int128 k = (__int128)hi - lo + 1;
    const __int128 target = k * 1000;
    __int128 mag = 1, v = 0;
    while (mag < target) {
        int32_t x = stdgen_next(g);
        v = v * b + (x - 1);
        mag *= b;
    }
    __int128 r = v % k;
    return lo + (int64_t)r;
}
