"""The wavefront-per-replica kernel at every near-queue depth it is built for
(K = 4, 24, 32 entries per lane: 256 / 1,536 / 2,048 events on chip) against
the oracle's canonical mode: the random tie-heavy programs, the tie audit's
probe orders (LIFO / scrambled seq keys, the case that once stalled a
K = 24 variant: DESIGN.md §3b), the reference's spec programs and a hotspot
whose receiver backlog overflows the smaller on-chip queues into the far
runs and heap (TimedT.hs:234-304, 357-368)."""
import numpy as np
import pytest

import progs
from timewarp import scenarios
from timewarp.abi import RESULT_FIELDS

pytestmark = [pytest.mark.gpu, pytest.mark.one_geometry]

KS = [4, 24, 32]


@pytest.fixture
def wave_k(request, monkeypatch):
    monkeypatch.setenv("TW_GEOMETRY", "wave")
    monkeypatch.setenv("TW_WAVE_K", str(request.param))
    return request.param


@pytest.mark.parametrize("wave_k", KS, indirect=True)
def test_random_programs_each_k(engine_mod, oracle_mod, wave_k):
    for seed in range(48):
        scn = progs.random_program(seed)
        with engine_mod.Engine(0) as e:
            e.load(scn)
            assert e.geometry() == "wave"
            e.run(t_end=3000)
            res, h = e.results(), e.hashes()
        o = oracle_mod.run(scn, t_end=3000)
        for f in RESULT_FIELDS:
            assert res[f][0] == o.result[f], (wave_k, seed, f, res[f][0], o.result[f])
        assert np.array_equal(h[0], o.hashes), (wave_k, seed)


@pytest.mark.parametrize("wave_k", KS, indirect=True)
def test_tie_audit_each_k(engine_mod, oracle_mod, wave_k):
    def same(a, b):
        return a.result == b.result and np.array_equal(a.hashes, b.hashes)

    for seed in range(16):
        scn = progs.random_program(seed)
        with engine_mod.Engine(0) as e:
            e.load(scn).tie_audit(probes=2, t_end=3000)
            res, h = e.results(), e.hashes()
        r = [oracle_mod.run(scn, mode=m, t_end=3000) for m in (0, 2, 3)]
        for f in RESULT_FIELDS:
            assert res[f][0] == r[0].result[f], (wave_k, seed, f)
        assert np.array_equal(h[0], r[0].hashes), (wave_k, seed)
        want = 1 | (0 if same(r[0], r[1]) else 2) | (0 if same(r[0], r[2]) else 4)
        assert int(res["tie_flags"][0]) == want, (wave_k, seed, int(res["tie_flags"][0]), want)


@pytest.mark.parametrize("wave_k", KS, indirect=True)
def test_spec_programs_each_k(engine_mod, oracle_mod, wave_k):
    for case in progs.KATS + progs.EXCEPTION_SPEC:
        scn, _ = case()
        st, res, h = engine_mod.run_scenario(scn)
        ores, oh = oracle_mod.run_batch(scn)
        for f in RESULT_FIELDS:
            assert np.array_equal(res[f], ores[f]), (wave_k, scn.name, f)
        assert np.array_equal(h, oh), (wave_k, scn.name)


@pytest.mark.parametrize("wave_k", KS, indirect=True)
def test_hotspot_backlog_each_k(engine_mod, oracle_mod, wave_k):
    # ~300 pings pending at the receiver: beyond 64 x 4 on chip at K = 4
    scn = scenarios.hotspot(n_senders=64, n_replicas=8, msg_num=60)
    st, res, h = engine_mod.run_scenario(scn)
    ores, oh = oracle_mod.run_batch(scn, threads=8)
    for f in RESULT_FIELDS:
        assert np.array_equal(res[f], ores[f]), (wave_k, f)
    assert np.array_equal(h, oh)
