"""ABI-2 semantics on the GPU, bit-exact against the oracle: handler stacks
deeper than the record (overflow frames), full-width exception payloads,
counter-wrap guard, tie-order audit flags, BinaryP transmission time at send,
and `close` resetting a connection's state."""
import numpy as np
import pytest

import progs
from timewarp import isa, scenarios
from timewarp.abi import RESULT_FIELDS
from timewarp.engine import Engine

pytestmark = pytest.mark.gpu


def _same(scn, res, h, ores, oh):
    for f in RESULT_FIELDS:
        assert np.array_equal(res[f], ores[f]), (scn.name, f, res[f][:4], ores[f][:4])
    assert np.array_equal(h, oh), scn.name


def _batch(scn, n):
    return scn.with_replicas(0, 1) if n == 1 else scn


@pytest.mark.parametrize("depth,max_frames", [(3, 8), (6, 8), (8, 8), (9, 8), (12, 14), (3, 0)])
def test_deep_handler_stack(engine_mod, oracle_mod, depth, max_frames):
    scn = progs.deep_catch_prog(depth, max_frames=max_frames, payload=(1 << 40) + 7)
    st, res, h = engine_mod.run_scenario(scn)
    ores, oh = oracle_mod.run_batch(scn)
    _same(scn, res, h, ores, oh)


@pytest.mark.parametrize("v", [(1 << 40) + 3, -(1 << 50) - 1, (1 << 63) - 1])
def test_full_width_payload_round_trips(engine_mod, oracle_mod, v):
    scn = progs.payload_prog(v)
    with Engine(0) as e:
        e.load(scn).set_trace(16).reset()
        e.run()
        recs, n = e.trace(0)
        res, h = e.results(), e.hashes()
    assert n == 1 and int(recs["val"][0]) == v
    ores, oh = oracle_mod.run_batch(scn)
    _same(scn, res, h, ores, oh)


def test_counter_wrap_is_a_status(engine_mod):
    scn = scenarios.token_ring(n_nodes=8, n_replicas=64, launch_duration=20_000_000)
    with Engine(0) as e:
        e.load(scn).set_counter_base(0xFFFFFFFF - 50, 1).reset()
        e.run()
        assert (e.results()["status"] == isa.REP_ERR_COUNTER).all()
        e.set_counter_base(0, 0xFFFFFFFF - 5).reset()
        e.run()
        assert (e.results()["status"] == isa.REP_ERR_COUNTER).all()


def test_counter_base_far_from_top_changes_nothing(engine_mod, oracle_mod):
    """seq and tid offsets are unobservable (tids never enter a hash)."""
    scn = scenarios.token_ring(n_nodes=8, n_replicas=64, launch_duration=20_000_000, drop_log2=3)
    with Engine(0) as e:
        e.load(scn).set_counter_base(1 << 31, 1 << 30).reset()
        e.run()
        res, h = e.results(), e.hashes()
    ores, oh = oracle_mod.run_batch(scn)
    _same(scn, res, h, ores, oh)


def test_tie_audit_flags_tie_sensitive_replicas(engine_mod, oracle_mod):
    """tw_tie_audit on tie-heavy random programs: a replica is flagged iff the
    oracle's probe modes give a different trace, and the canonical results that
    stay loaded equal the oracle's canonical run."""
    def same(a, b):
        return a.result == b.result and np.array_equal(a.hashes, b.hashes)

    flagged = 0
    for seed in range(16):
        scn = progs.random_program(seed)
        with Engine(0) as e:
            e.load(scn).tie_audit(probes=2, t_end=3000)
            res, h = e.results(), e.hashes()
        r = [oracle_mod.run(scn, mode=m, t_end=3000) for m in (0, 2, 3)]
        for f in RESULT_FIELDS:
            assert res[f][0] == r[0].result[f], (seed, f)
        assert np.array_equal(h[0], r[0].hashes), seed
        want = 1 | (0 if same(r[0], r[1]) else 2) | (0 if same(r[0], r[2]) else 4)
        assert int(res["tie_flags"][0]) == want, (seed, int(res["tie_flags"][0]), want)
        flagged += want != 1
    assert flagged > 0


def test_tie_audit_configs_insensitive(engine_mod):
    scn = scenarios.token_ring(n_nodes=16, n_replicas=128, launch_duration=30_000_000, drop_log2=3)
    with Engine(0) as e:
        e.load(scn).tie_audit(probes=2)
        assert (e.results()["tie_flags"] == 1).all()


def test_binaryp_transmission_time_on_device(engine_mod, oracle_mod):
    scn = scenarios.hotspot(n_senders=8, n_replicas=64, msg_num=40)
    scn.msg_bytes = np.array([37, 1234], np.uint32)
    scn.link_bw = (np.arange(scn.topo.n_links, dtype=np.uint64) % 5 + 1) * 100_000
    st, res, h = engine_mod.run_scenario(scn)
    ores, oh = oracle_mod.run_batch(scn)
    _same(scn, res, h, ores, oh)


def test_close_resets_connection_state(engine_mod, oracle_mod):
    scn = scenarios.socket_state(n_replicas=64, close_every=2)
    st, res, h = engine_mod.run_scenario(scn)
    ores, oh = oracle_mod.run_batch(scn)
    _same(scn, res, h, ores, oh)
