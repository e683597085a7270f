"""Config 4 (single gossip scenario, node-partitioned, lookahead windows):
the LP engine with P contexts must equal the sequential TimedT oracle on every
counter and every node hash ("run the node-partitioned engine with P
logical shards on 1 GPU and require the results to equal the P=1 run")."""
import numpy as np
import pytest

from timewarp import scenarios

pytestmark = pytest.mark.gpu

FIELDS = ["final_t", "events", "delivered", "dropped", "undeliverable", "status", "main_exc", "threads"]


@pytest.mark.one_geometry  # LP mode: the replica geometries do not apply
@pytest.mark.parametrize("n,parts,drop", [(64, 1, 0), (1000, 1, 0), (1000, 4, 0), (5000, 3, 4), (50000, 8, 0)])
def test_gossip_partitioned_equals_oracle(engine_mod, oracle_mod, n, parts, drop):
    scn = scenarios.gossip(n, drop_log2=drop, seed=n)
    agg, hashes, windows = engine_mod.run_partitioned(scn, parts=parts)
    o = oracle_mod.run(scn, trace_cap=0)
    for f in FIELDS:
        assert int(agg[f]) == int(o.result[f]), (f, int(agg[f]), o.result[f])
    assert np.array_equal(hashes, o.hashes)
    assert windows > 1


@pytest.mark.one_geometry  # LP mode: the replica geometries do not apply
@pytest.mark.parametrize("parts", [1, 4])
def test_gossip_inline_handlers_partitioned(engine_mod, oracle_mod, parts):
    """In-place handler dispatch (MonadDialog.hs:114-117) on the LP engine: the
    phantom deliverer runs the handler itself."""
    scn = scenarios.gossip(3000, seed=11, fork_strategy="inline")
    agg, hashes, windows = engine_mod.run_partitioned(scn, parts=parts)
    o = oracle_mod.run(scn, trace_cap=0)
    for f in FIELDS:
        assert int(agg[f]) == int(o.result[f]), (f, int(agg[f]), o.result[f])
    assert np.array_equal(hashes, o.hashes)


def test_gossip_replica_engine(engine_mod, oracle_mod):
    """The same scenario as one replica on the replica engine."""
    scn = scenarios.gossip(2000, seed=5)
    st, res, h = engine_mod.run_scenario(scn)
    o = oracle_mod.run(scn, trace_cap=0)
    for f in FIELDS:
        assert int(res[f][0]) == int(o.result[f]), f
    assert np.array_equal(h[0], o.hashes)


@pytest.mark.one_geometry  # LP mode: the replica geometries do not apply
def test_lookahead_violation_is_an_error(engine_mod):
    """token-ring's observer links have 0 µs delay (examples/token-ring/Main.hs:75-76):
    no conservative window exists, and the LP engine must say so instead of
    producing a wrong trace."""
    from timewarp import isa

    scn = scenarios.token_ring(n_nodes=8, n_replicas=1, launch_duration=20_000_000)
    agg, hashes, windows = engine_mod.run_partitioned(scn, parts=2, lookahead_us=1000, max_windows=100000)
    assert int(agg["status"]) == isa.REP_ERR_INSN


@pytest.mark.one_geometry
@pytest.mark.parametrize("n,parts,drop", [(1000, 1, 0), (5000, 3, 4), (50000, 8, 0)])
def test_gossip_device_windows_equal_oracle(engine_mod, oracle_mod, n, parts, drop):
    """The device-driven window loop (tw_lp_tick / tw_lp_run_windows: the
    window start, the work lists and the record exchange stay on the device)
    gives the sequential oracle's counters and node hashes, and runs the same
    windows as the host-driven loop."""
    scn = scenarios.gossip(n, drop_log2=drop, seed=n)
    agg, hashes, windows, ticks = engine_mod.run_partitioned_device(scn, parts=parts)
    o = oracle_mod.run(scn, trace_cap=0)
    for f in FIELDS:
        assert int(agg[f]) == int(o.result[f]), (f, int(agg[f]), o.result[f])
    assert np.array_equal(hashes, o.hashes)
    _, _, host_windows = engine_mod.run_partitioned(scn, parts=parts)
    # a window after one whose lanes delivered records straight into inboxes
    # starts at that window's end (a bound below every such record) rather than
    # at the earliest record: at most one extra, empty window per window
    assert host_windows <= windows <= 2 * host_windows and ticks >= windows


@pytest.mark.one_geometry
@pytest.mark.parametrize("parts", [1, 3])
def test_gossip_device_windows_rerun_ticks(engine_mod, oracle_mod, monkeypatch, parts):
    """Windows that take several ticks (a lane budget of 2 pops per tick): the
    device loop reruns the window, drains inboxes only at its first tick, and
    the result is still the oracle's."""
    monkeypatch.setenv("TW_LP_TICK_BUDGET", "2")
    scn = scenarios.gossip(3000, drop_log2=4, seed=7)
    agg, hashes, windows, ticks = engine_mod.run_partitioned_device(scn, parts=parts)
    o = oracle_mod.run(scn, trace_cap=0)
    for f in FIELDS:
        assert int(agg[f]) == int(o.result[f]), (f, int(agg[f]), o.result[f])
    assert np.array_equal(hashes, o.hashes)
    assert ticks > windows


@pytest.mark.one_geometry
def test_gossip_device_windows_inbox_overflow_is_an_error(engine_mod, oracle_mod):
    """An inbox of one record per node: a node sent more than that in a window
    ends the device loop with TW_ERR_REPLICA (the drain keeps to the capacity,
    never reading another node's records), and the device stays usable."""
    scn = scenarios.gossip(2000, seed=3)
    s = engine_mod.lp_scenario(scn)
    e = engine_mod.LPEngine(s, 0, scn.n_nodes, int(scn.meta["lookahead_us"]), 0, inbox_cap=1)
    try:
        e.reset()
        e.loop_begin()
        with pytest.raises(engine_mod.EngineError, match=r"failed: -6 "):
            e.run_windows(1 << 20)
    finally:
        e.close()
    agg, hashes, windows, ticks = engine_mod.run_partitioned_device(scn, parts=1)
    o = oracle_mod.run(scn, trace_cap=0)
    for f in FIELDS:
        assert int(agg[f]) == int(o.result[f]), (f, int(agg[f]), o.result[f])
    assert np.array_equal(hashes, o.hashes)
