"""The engine under the tie orders besides the canonical one, against the
oracle in the same order, every output field and node hash bit-exact, under
every replica geometry: TW_TIE_LIFO (equal timestamps in reverse insertion
order, oracle mode 2) and TW_TIE_FORKFIRST (FIFO, but a forked child is always
the next pop, oracle mode 5).

Under both a fork's child is always the next pop -- as under TimedT's own
pqueue MinQueue, where an insert whose key is <= the held minimum's becomes
the minimum (TimedT.hs:242, 326-342) -- so the replica kernels run it in
place (Lane::fork_in_place); these cases pin that path: the child's thread
id, slot, insertion counter value, pop count, clock and hash term, the
parent's queue entry and record, forks in a row (grand-children), forks onto
other nodes, deliverer forks (send), handler forks (deliver) and the
timeout watchdog's fork.  The BASELINE scenarios come out identical to the
canonical order too (they are tie-insensitive)."""
import numpy as np
import pytest

import progs
from timewarp import scenarios
from timewarp.abi import RESULT_FIELDS
from timewarp.engine import Engine

pytestmark = [pytest.mark.gpu, pytest.mark.one_geometry]

FIELDS = [f for f in RESULT_FIELDS if f != "tie_flags"]
ORACLE_MODE = {"lifo": 2, "forkfirst": 5}  # oracle MODE_LIFO, MODE_FORKFIRST


@pytest.fixture(params=["lifo", "forkfirst"])
def order(request):
    return request.param


def _gpu(scn, order, t_end=None, geo="dense"):
    with Engine(0) as e:
        e.load(scn, geometry=geo)
        if order == "forkfirst" and e.geometry() == "wave":
            pytest.skip("TW_TIE_FORKFIRST: lane-per-replica geometries")
        e.set_tie_mode(order).reset()
        st = e.run() if t_end is None else e.run(t_end)
        return st, e.results(), e.hashes()


def _check(scn, oracle_mod, order, t_end=None, canonical_too=False, geo="dense"):
    st, res, h = _gpu(scn, order, t_end, geo)
    mode = ORACLE_MODE[order]
    if t_end is None:
        ores, oh = oracle_mod.run_batch(scn, mode=mode, threads=8)
        for f in FIELDS:
            assert np.array_equal(res[f], ores[f]), (scn.name, f, res[f][:4], ores[f][:4])
        assert np.array_equal(h, oh), scn.name
    else:
        for r in range(scn.n_replicas):
            o = oracle_mod.run(scn, replica=r, mode=mode, t_end=t_end)
            for f in FIELDS:
                assert res[f][r] == o.result[f], (scn.name, r, f, res[f][r], o.result[f])
            assert np.array_equal(h[r], o.hashes), (scn.name, r)
    if canonical_too:  # a tie-insensitive scenario: the canonical order's results
        cres, ch = oracle_mod.run_batch(scn, threads=8)
        for f in FIELDS:
            assert np.array_equal(res[f], cres[f]), (scn.name, "canonical", f)
        assert np.array_equal(h, ch), (scn.name, "canonical")
    return st, res


@pytest.mark.parametrize("seed", range(0, 48, 6))
def test_random_programs(engine_mod, oracle_mod, order, seed):
    _check(progs.random_program(seed), oracle_mod, order, t_end=3000)


def test_spec_programs(engine_mod, oracle_mod, order):
    for case in progs.KATS + progs.EXCEPTION_SPEC:
        scn, _ = case()
        _check(scn, oracle_mod, order)


@pytest.mark.parametrize("tout,wt", [(0, 0), (2, 1), (10, 5), (3, 3)])
def test_timeout(engine_mod, oracle_mod, order, tout, wt):
    _check(progs.timeout_prog(tout, wt), oracle_mod, order)


@pytest.mark.parametrize("geo", ["dense", "compact", "narrow", "sparse", "half"])
def test_token_ring(engine_mod, oracle_mod, order, geo):
    scn = scenarios.token_ring(n_nodes=12, n_replicas=300, launch_duration=200_000_000, drop_log2=4, link_depth=8)
    _, res = _check(scn, oracle_mod, order, canonical_too=True, geo=geo)
    assert res["dropped"].sum() > 0


@pytest.mark.parametrize("geo", ["dense", "narrow"])
def test_token_ring_c3_shape(engine_mod, oracle_mod, order, geo):
    # C3's shape: main's 4,096 forks, every node's worker/server/killer forks
    scn = scenarios.token_ring(n_nodes=4096, n_replicas=8, launch_duration=120_000_000, drop_log2=10)
    _check(scn, oracle_mod, order, canonical_too=True, geo=geo)


@pytest.mark.parametrize("geo", ["compact", "dense"])
def test_ping_pong(engine_mod, oracle_mod, order, geo):
    _check(scenarios.ping_pong(n_replicas=500, round_trips=40), oracle_mod, order, canonical_too=True, geo=geo)


@pytest.mark.parametrize("geo", ["sparse", "narrow"])
def test_hotspot(engine_mod, oracle_mod, order, geo):
    _check(scenarios.hotspot(n_senders=8, n_replicas=64, msg_num=30), oracle_mod, order, canonical_too=True, geo=geo)


def test_gatekeeper(engine_mod, oracle_mod, order):
    _check(scenarios.gatekeeper(n_clients=6, n_replicas=100, msg_num=24, junk_every=3), oracle_mod, order)
