"""TimedT's own equal-timestamp order on the GPU (tw_set_tie_mode(PQUEUE)).

`Event`'s `Ord` compares timestamps only (TimedT.hs:100-104), so the order of
equal-timestamp events is whatever pqueue-1.3.1.1's binomial MinQueue gives
(TimedT.hs:242), and every throwTo rebuilds the queue with
`fromList . map . toList` (TimedT.hs:361-368).  In this mode the wavefront-
per-replica kernel keeps each replica's queue as that MinQueue; a replica the
tie audit flags can be re-run in TimedT's order.  The reference point is the
oracle's pqueue mode (mode 1: oracle/pqueue_min.hpp); pqueue itself is not in
the reference, so this order is PARITY UNPINNED beyond that transcription."""
import numpy as np
import pytest

import progs
from timewarp import scenarios
from timewarp.abi import RESULT_FIELDS

pytestmark = [pytest.mark.gpu, pytest.mark.one_geometry]


def _gpu_pq(engine_mod, scn, t_end=None):
    with engine_mod.Engine(0) as e:
        e.load(scn, geometry="wave")
        e.set_tie_mode("pqueue").reset()
        if t_end is None:
            e.run()
        else:
            e.run(t_end=t_end)
        return e.results(), e.hashes()


def _check(res, h, o, tag, i=0):
    for f in RESULT_FIELDS:
        if f == "tie_flags":
            continue
        assert res[f][i] == o.result[f], (tag, f, res[f][i], o.result[f])
    assert np.array_equal(h[i], o.hashes), tag


def test_random_programs_in_pqueue_order(engine_mod, oracle_mod):
    """The 48 tie-heavy random programs: GPU pqueue mode == oracle mode 1,
    field by field and node hash by node hash -- including the ones whose
    outputs differ between the canonical and the pqueue order."""
    differ = 0
    for seed in range(48):
        scn = progs.random_program(seed)
        res, h = _gpu_pq(engine_mod, scn, t_end=3000)
        o1 = oracle_mod.run(scn, mode=1, t_end=3000)
        _check(res, h, o1, seed)
        o0 = oracle_mod.run(scn, mode=0, t_end=3000)
        differ += not (o0.result == o1.result and np.array_equal(o0.hashes, o1.hashes))
    assert differ > 0  # some programs do depend on the tie order


def test_spec_programs_in_pqueue_order(engine_mod, oracle_mod):
    for case in progs.KATS + progs.EXCEPTION_SPEC:
        scn, _ = case()
        res, h = _gpu_pq(engine_mod, scn)
        for r in range(scn.n_replicas):
            o1 = oracle_mod.run(scn, mode=1, replica=r)
            _check(res, h, o1, scn.name, r)


@pytest.mark.parametrize("tout,wt", [(1, 0), (2, 1), (7, 6), (3, 3)])
def test_timeout_ties_in_pqueue_order(engine_mod, oracle_mod, tout, wt):
    # `timeout` with tout == wt + 1 sits exactly on a tie
    scn = progs.timeout_prog(tout, wt)
    res, h = _gpu_pq(engine_mod, scn)
    _check(res, h, oracle_mod.run(scn, mode=1), (tout, wt))


def test_token_ring_in_pqueue_order(engine_mod, oracle_mod):
    # a BASELINE scenario with throwTo on every hop (the rebuild path)
    scn = scenarios.token_ring(n_nodes=8, n_replicas=6, launch_duration=20_000_000, drop_log2=3)
    res, h = _gpu_pq(engine_mod, scn)
    for r in range(scn.n_replicas):
        _check(res, h, oracle_mod.run(scn, mode=1, replica=r), "token_ring", r)


def test_token_ring_c3_nodes_in_pqueue_order(engine_mod, oracle_mod):
    # C3's 4,096 nodes: by 10.5 s the queue holds ~12k events (every node's
    # sleeping worker and server, its killer at launchDuration) and each token
    # hop's throwTo rebuilds all of it (TimedT.hs:361-368).  Cut at 10.5 s
    # (start-up + the first hops): the teardown's 8,192 rebuilds in the wave
    # kernel's scalar MinQueue would take minutes
    scn = scenarios.token_ring(n_nodes=4096, n_replicas=1, launch_duration=120_000_000, drop_log2=10)
    t_end = 10_500_000
    res, h = _gpu_pq(engine_mod, scn, t_end=t_end)
    o = oracle_mod.run(scn, mode=1, replica=0, t_end=t_end)
    _check(res, h, o, "token_ring_4096")
    assert o.result["delivered"] >= 3 and o.result["events"] > 30_000


def test_token_ring_teardown_in_pqueue_order(engine_mod, oracle_mod):
    # the whole launchDuration, teardown included: at 120 s each of the 512
    # kill pairs throws twice and every throwTo rebuilds the ~1.5k-entry queue
    # with `fromList . map . toList` (TimedT.hs:361-368; examples/token-ring/
    # Main.hs:124-127), against the oracle's pqueue transcription (mode 1)
    scn = scenarios.token_ring(n_nodes=512, n_replicas=2, launch_duration=120_000_000, drop_log2=10)
    res, h = _gpu_pq(engine_mod, scn)
    for r in range(scn.n_replicas):
        o = oracle_mod.run(scn, mode=1, replica=r)
        _check(res, h, o, "token_ring_512_teardown", r)
        assert o.result["final_t"] == 120_000_000 and o.result["status"] == 1


def test_pqueue_mode_needs_the_wave_geometry(engine_mod):
    scn = progs.random_program(0)
    with engine_mod.Engine(0) as e:
        e.load(scn, geometry="dense")
        with pytest.raises(engine_mod.EngineError, match=r"failed: -1 "):
            e.set_tie_mode("pqueue")
