"""Third-party arithmetic on the path, both un-vendored:

* pqueue-1.3.1.1 Data.PQueue.Min (stack.yaml:21) — the C++ transcription
  (oracle/pqueue_min.hpp) is cross-checked against a second, literal
  recursive Python transcription of the published Haskell code below
  (persistent BinomForest with Skip/Cons, extractBin/incrExtract/incrExtract').
  PARITY UNPINNED against pqueue itself: no reference test fixes tie order.
* random-1.1 StdGen — the product's numpy generator (timewarp/stdgen.py) and
  the oracle's C++ one (oracle/stdgen.hpp) are independent restatements;
  pinned by hand-derived values of the published algorithm.
"""
from collections import namedtuple

import numpy as np
import pytest

from timewarp.stdgen import StdGenVec

# ----------------------------------------------- literal pqueue transcription
Extract = namedtuple("Extract", "min_key children forest")


def _le(a, b):
    return a[0] <= b[0]


def _join(t1, t2):  # joinBin le t1 t2
    (x1, c1), (x2, c2) = t1, t2
    return (x1, (t2,) + c1) if _le(x1, x2) else (x2, (t1,) + c2)


def _incr(t, f):  # incr le t f   (f: tuple, index = rank offset; None = Skip)
    if not f:
        return (t,)
    if f[0] is None:
        return (t,) + f[1:]
    return (None,) + _incr(_join(t, f[0]), f[1:])


def _extract_bin(f):
    if not f:
        return None
    head, rest = f[0], f[1:]
    if head is None:
        ex = _extract_bin(rest)
        if ex is None:
            return None
        # incrExtract: Extract k (Succ kChild kChildren) ts -> Extract k kChildren (Cons kChild ts)
        return Extract(ex.min_key, ex.children[1:], (ex.children[0],) + ex.forest)
    x, ts = head
    ex = _extract_bin(rest)
    if ex is not None and not _le(x, ex.min_key):  # x' `lt` x
        # incrExtract': Skip (incr (t `joinBin` kChild) ts)
        return Extract(ex.min_key, ex.children[1:], (None,) + _incr(_join(head, ex.children[0]), ex.forest))
    return Extract(x, ts, (None,) + rest)


class HsMinQueue:
    def __init__(self):
        self.q = None  # (n, xmin, forest)

    def insert(self, x):
        if self.q is None:
            self.q = (1, x, ())
            return
        n, m, f = self.q
        if _le(x, m):
            self.q = (n + 1, x, _incr((m, ()), f))
        else:
            self.q = (n + 1, m, _incr((x, ()), f))

    def pop(self):
        n, m, f = self.q
        ex = _extract_bin(f)
        self.q = None if ex is None else (n - 1, ex.min_key, ex.forest)
        return m


def _hs_order(ops):
    q, out = HsMinQueue(), []
    for i, k in enumerate(ops):
        if k >= 0:
            q.insert((k, i))
        elif q.q is not None:
            out.append(q.pop()[1])
    return out


def test_pqueue_pure_ties_are_lifo(oracle_mod):
    """insert x <= xmin makes x the held min: equal keys inserted in sequence pop LIFO."""
    assert oracle_mod.pqueue_order([5] * 6 + [-1] * 6).tolist() == [5, 4, 3, 2, 1, 0]


@pytest.mark.parametrize("seed", range(40))
def test_pqueue_matches_literal_transcription(oracle_mod, seed):
    rng = np.random.default_rng(seed)
    n = int(rng.integers(5, 400))
    keys = rng.integers(0, int(rng.choice([2, 4, 16, 1000])), size=n)
    pops = rng.random(n) < 0.4
    ops = np.where(pops, -1, keys).tolist() + [-1] * n
    cxx = oracle_mod.pqueue_order(ops).tolist()
    assert cxx == _hs_order(ops)
    # and it is a valid priority queue: popped keys never decrease between inserts
    assert len(cxx) == sum(1 for k in ops if k >= 0)


def test_pqueue_rebuild_roundtrip(oracle_mod):
    """fromList . toList keeps the pop order (TimedT.hs:368 with no key change)."""
    rng = np.random.default_rng(7)
    keys = rng.integers(0, 5, size=200).tolist()
    q = HsMinQueue()
    for i, k in enumerate(keys):
        q.insert((k, i))
    asc = []
    while q.q is not None:
        asc.append(q.pop())
    q2 = HsMinQueue()
    for x in reversed(asc):  # foldr insert empty
        q2.insert(x)
    again = []
    while q2.q is not None:
        again.append(q2.pop())
    assert again == asc


# ----------------------------------------------------------------- StdGen
def test_stdgen_hand_derived():
    """mkStdGen 0 = StdGen 1 1; next -> 40014 - 40692 + 2147483562 = 2147482884;
    randomR (1000, 5000) -> 1000 + 2147482883 mod 4001 = 3147."""
    g = StdGenVec([0])
    assert int(g.s1[0]) == 1 and int(g.s2[0]) == 1
    assert int(g.next()[0]) == 2147482884
    assert int(StdGenVec([0]).range(1000, 5000)[0]) == 3147


@pytest.mark.parametrize("seed", [0, 1, 42, -1, 2**31 - 1, 2**31, 2**40 + 5, -(2**35), 123456789])
def test_stdgen_python_vs_cpp(oracle_mod, seed):
    (s1, s2), nxt = oracle_mod.stdgen_next(seed, 64)
    g = StdGenVec([seed])
    assert (int(g.s1[0]), int(g.s2[0])) == (s1, s2)
    assert [int(g.next()[0]) for _ in range(64)] == nxt.tolist()
    for lo, hi in [(1000, 5000), (0, 1023), (0, 1), (7, 7)]:
        g = StdGenVec([seed])
        assert [int(g.range(lo, hi)[0]) for _ in range(32)] == oracle_mod.stdgen_draws(seed, lo, hi, 32).tolist()


def test_stdgen_vectorised_over_replicas():
    seeds = np.arange(1000, dtype=np.int64)
    g = StdGenVec(seeds)
    a = g.range(1000, 5000)
    b = np.array([int(StdGenVec([s]).range(1000, 5000)[0]) for s in seeds])
    assert np.array_equal(a, b)
    assert a.min() >= 1000 and a.max() <= 5000
