"""random-1.1 ``StdGen`` vectorised over replicas (host-side table drawing).

The reference draws network delays with ``mkStdGen 0`` and ``getRandomTR``
(examples/token-ring/Main.hs:9,60,77).  random-1.1 is an un-vendored
dependency (lts-7.9, time-warp.cabal:69); this restates its published
algorithm:

  mkStdGen s  : s' = s .&. 0x7fffffff (after Int -> Int32); (q, s1) = s' divMod
                2147483562; s2 = q mod 2147483398; StdGen (s1+1) (s2+1)
  next        : L'Ecuyer combined MLCG, output z in [1, 2147483562]
  randomR     : randomIvalInteger — for ranges k <= 2147483 one `next`:
                lo + (x-1) mod k

Every draw of the engine's link tables comes from here, so GPU traces are
deterministic and identical to the oracle's (which restates the same
algorithm independently in oracle/stdgen.hpp; tests cross-check the two).
"""
from __future__ import annotations

import numpy as np


class StdGenVec:
    """R independent generators, one per replica, stepped in lock-step."""

    def __init__(self, seeds):
        s = np.asarray(seeds, dtype=np.int64)
        s32 = (s & 0xFFFFFFFF).astype(np.uint32).view(np.int32).astype(np.int64)
        s31 = s32 & 0x7FFFFFFF
        q, s1 = np.divmod(s31, 2147483562)
        s2 = q % 2147483398
        self.s1 = (s1 + 1).astype(np.int64)
        self.s2 = (s2 + 1).astype(np.int64)

    def next(self) -> np.ndarray:
        s1, s2 = self.s1, self.s2
        k = s1 // 53668  # s1 > 0: quot == div
        s1 = 40014 * (s1 - k * 53668) - k * 12211
        s1 = np.where(s1 < 0, s1 + 2147483563, s1)
        k2 = s2 // 52774
        s2 = 40692 * (s2 - k2 * 52774) - k2 * 3791
        s2 = np.where(s2 < 0, s2 + 2147483399, s2)
        self.s1, self.s2 = s1, s2
        z = s1 - s2
        return np.where(z < 1, z + 2147483562, z)

    def range(self, lo: int, hi: int) -> np.ndarray:
        """``randomR (lo, hi)`` for Integer ranges needing a single ``next``."""
        if lo > hi:
            lo, hi = hi, lo
        k = hi - lo + 1
        if k * 1000 > 2147483562:
            raise ValueError("range needs more than one StdGen digit; not used by any config")
        x = self.next()
        return lo + (x - 1) % k


def stdgen_draws(seed: int, lo: int, hi: int, n: int) -> np.ndarray:
    g = StdGenVec([seed])
    return np.array([int(g.range(lo, hi)[0]) for _ in range(n)], dtype=np.int64)
