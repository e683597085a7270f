"""Full-shape parity: the BASELINE configs at their real
per-replica shape, few replicas each, GPU vs oracle field by field and node
hash by node hash.
  C3  examples/token-ring/Main.hs:104-154 at 4,096 nodes, delay+drop nastiness
  C5  bench/Network Sender/Main.hs:34-64 + Receiver/Main.hs:32-41 with all 256
      senders on one receiver (the skewed hotspot: a deep receiver backlog)
  C4  one gossip scenario of 2^20 nodes, 8 logical shards (node partitioning)"""
import numpy as np
import pytest

from timewarp import scenarios
from timewarp.abi import RESULT_FIELDS

pytestmark = pytest.mark.gpu


def _compare(engine_mod, oracle_mod, scn):
    st, res, h = engine_mod.run_scenario(scn)
    ores, oh = oracle_mod.run_batch(scn, threads=16)
    for f in RESULT_FIELDS:
        assert np.array_equal(res[f], ores[f]), (scn.name, f, res[f][:4], ores[f][:4])
    assert np.array_equal(h, oh), scn.name
    return res


def test_c3_token_ring_4096_nodes(engine_mod, oracle_mod):
    scn = scenarios.token_ring(n_nodes=4096, n_replicas=64, launch_duration=120_000_000, drop_log2=10)
    res = _compare(engine_mod, oracle_mod, scn)
    assert int(res["events"].min()) > 40_000


def test_c3_token_ring_full_lap_with_drops(engine_mod, oracle_mod):
    """launchDuration beyond a full lap (the messaging-dominated shape) with
    frequent drops, so the token dies and the checker logs no-progress."""
    scn = scenarios.token_ring(n_nodes=512, n_replicas=32, launch_duration=1_700_000_000, drop_log2=6,
                               link_depth=4)
    res = _compare(engine_mod, oracle_mod, scn)
    assert int(res["dropped"].sum()) > 0 and int(res["delivered"].sum()) > 1000


def test_c5_hotspot_256_senders(engine_mod, oracle_mod):
    scn = scenarios.hotspot(n_senders=256, n_replicas=16, msg_num=100)
    res = _compare(engine_mod, oracle_mod, scn)
    assert int(res["delivered"].min()) > 256 * 100


_C4 = {}


def _c4_oracle(oracle_mod):
    """The sequential oracle's run of BASELINE config 4 (one gossip scenario of
    2^20 nodes), computed once for the tests below."""
    if "o" not in _C4:
        _C4["scn"] = scenarios.gossip(1 << 20, seed=0)
        _C4["o"] = oracle_mod.run(_C4["scn"], trace_cap=0)
    return _C4["scn"], _C4["o"]


@pytest.mark.one_geometry
def test_c4_gossip_1m_nodes_8_shards(engine_mod, oracle_mod):
    scn, o = _c4_oracle(oracle_mod)
    agg, hashes, windows = engine_mod.run_partitioned(scn, parts=8)
    for f in RESULT_FIELDS:
        assert int(agg[f]) == int(o.result[f]), (f, int(agg[f]), o.result[f])
    assert np.array_equal(hashes, o.hashes)
    assert windows > 10


@pytest.mark.one_geometry
@pytest.mark.parametrize("parts", [1, 8])
def test_c4_gossip_1m_nodes_device_loop(engine_mod, oracle_mod, parts):
    """The path bench.py times for C4: the device-driven window loop
    (tw_lp_tick / tw_lp_tick_import / tw_lp_tick_end) at the full 2^20 nodes,
    as one context and as 8 logical shards exchanging record blocks, against
    the sequential oracle field by field and node hash by node hash
    (MonadDialog.hs:149-166 send path, TimedT.hs:234-304 loop)."""
    scn, o = _c4_oracle(oracle_mod)
    agg, hashes, windows, ticks = engine_mod.run_partitioned_device(scn, parts=parts)
    for f in RESULT_FIELDS:
        assert int(agg[f]) == int(o.result[f]), (f, parts, int(agg[f]), o.result[f])
    assert np.array_equal(hashes, o.hashes)
    assert windows > 10 and ticks >= windows


@pytest.mark.one_geometry
def test_c5_lpb_full_backlog(engine_mod, oracle_mod):
    """The path bench.py times for C5 (geometry lpb) at the real per-replica
    shape: 256 senders x 1,000 pings each at 1,000/s onto one receiver
    (bench/Network/Sender/Main.hs:34-64, Receiver/Main.hs:32-41), so the
    receiver's backlog runs to ~1.1-1.8k pending records through tw_lp_due
    every window; 4 replicas against the oracle's sequential runs, every
    result field and every node hash."""
    scn = scenarios.hotspot(n_senders=256, n_replicas=4, msg_num=1000)
    with engine_mod.Engine(0) as e:
        e.load(scn, geometry="lpb")
        assert e.geometry() == "lpb"
        e.reset()
        st = e.run()
        res, hashes = e.results(), e.hashes()
    ores, ohashes = oracle_mod.run_batch(scn, threads=4)
    for f in RESULT_FIELDS:
        if f != "tie_flags":
            assert np.array_equal(res[f], ores[f]), (f, res[f], ores[f])
    assert np.array_equal(hashes, ohashes)
    assert st.events == int(ores["events"].sum())
    assert int(ores["delivered"].min()) == 2 * 256 * 1000
