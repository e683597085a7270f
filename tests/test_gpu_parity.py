"""GPU engine vs oracle (canonical mode): bit-exact on every output.

Runs through the C ABI (libtimewarp.so) on cuda:0; no torch involved.  The
oracle is the CPU restatement of TimedT (oracle/timedt_oracle.cpp)."""
import numpy as np
import pytest

from timewarp import scenarios
from timewarp.abi import RESULT_DTYPE, RESULT_FIELDS

pytestmark = pytest.mark.gpu

FIELDS = list(RESULT_FIELDS)


def _compare(scn, engine_mod, oracle_mod, threads=8):
    st, res, hashes = engine_mod.run_scenario(scn)
    ores, ohashes = oracle_mod.run_batch(scn, threads=threads)
    bad = {}
    for f in FIELDS:
        m = np.nonzero(res[f] != ores[f])[0]
        if m.size:
            bad[f] = (m[:5].tolist(), res[f][m[:5]].tolist(), ores[f][m[:5]].tolist())
    hm = np.nonzero((hashes != ohashes).any(axis=1))[0]
    if hm.size:
        bad["hashes"] = hm[:5].tolist()
    assert not bad, f"{scn.name}: GPU != oracle: {bad}"
    assert st.events == int(ores["events"].sum())
    return st, ores


def test_token_ring_small(engine_mod, oracle_mod):
    scn = scenarios.token_ring(n_nodes=16, n_replicas=256, launch_duration=20_000_000)
    st, ores = _compare(scn, engine_mod, oracle_mod)
    assert (ores["status"] == 1).all()


def test_token_ring_drop_long(engine_mod, oracle_mod):
    scn = scenarios.token_ring(n_nodes=12, n_replicas=300, launch_duration=200_000_000, drop_log2=4,
                               link_depth=8)
    st, ores = _compare(scn, engine_mod, oracle_mod)
    assert ores["dropped"].sum() > 0


def test_ping_pong(engine_mod, oracle_mod):
    scn = scenarios.ping_pong(n_replicas=1000, round_trips=50)
    _compare(scn, engine_mod, oracle_mod)


def test_hotspot_small(engine_mod, oracle_mod):
    scn = scenarios.hotspot(n_senders=8, n_replicas=130, msg_num=40)
    _compare(scn, engine_mod, oracle_mod)


def test_gatekeeper_raw_listener(engine_mod, oracle_mod):
    """listenR (MonadDialog.hs:226-256): the raw listener runs for every
    message (also `Junk`, which has no typed listener) and gates the typed one."""
    scn = scenarios.gatekeeper(n_clients=6, n_replicas=200, msg_num=24, junk_every=3)
    st, ores = _compare(scn, engine_mod, oracle_mod)
    assert (ores["status"] == 1).all() and ores["undeliverable"].sum() == 0


def test_socket_state_user_state(engine_mod, oracle_mod):
    """examples/socket-state: per-connection `userStateR` counters (state cells
    addressed by the incoming link) and the server's stop at 10 s."""
    scn = scenarios.socket_state(n_replicas=300, seed_base=7)
    st, ores = _compare(scn, engine_mod, oracle_mod)
    assert (ores["status"] == 1).all() and ores["undeliverable"].sum() > 0


def test_hotspot_inline_handlers(engine_mod, oracle_mod):
    """ForkStrategy `const id` (MonadDialog.hs:114-117): Ping and Pong handlers
    run in place in the delivering thread, on the destination node."""
    scn = scenarios.hotspot(n_senders=8, n_replicas=130, msg_num=40, fork_strategy="inline")
    st, ores = _compare(scn, engine_mod, oracle_mod)
    assert ores["delivered"].sum() > 0


def test_hotspot_trace_records_and_measures(engine_mod, oracle_mod):
    """TRACE records (tw_set_trace / tw_read_trace) equal the oracle's trace log
    record for record, so measures.csv (bench/Network/LogReader/Main.hs:85-119)
    built from the GPU run is the oracle's."""
    from timewarp.measures import format_measures_csv, measures_from_trace, trace_tuples

    scn = scenarios.hotspot(n_senders=6, n_replicas=70, msg_num=12)
    with engine_mod.Engine() as e:
        e.load(scn)
        e.set_trace(1 << 11)
        e.reset()
        e.run()
        for rep in (0, 33, 69):
            recs, n = e.trace(rep)
            o = oracle_mod.run(scn, replica=rep, trace_cap=1 << 11)
            assert n == len(o.traces) == len(recs) > 0
            assert trace_tuples(recs) == trace_tuples(o.traces)
            assert format_measures_csv(measures_from_trace(trace_tuples(recs))) == \
                format_measures_csv(measures_from_trace(trace_tuples(o.traces)))
        # a small capacity keeps the first records and still counts the rest
        e.set_trace(5)
        e.reset()
        e.run()
        recs, n = e.trace(7)
        o = oracle_mod.run(scn, replica=7, trace_cap=1 << 11)
        assert len(recs) == 5 and n == len(o.traces)
        assert trace_tuples(recs) == trace_tuples(o.traces)[:5]


def test_hotspot_bandwidth_aware_delays(engine_mod, oracle_mod):
    """Link delays carrying the BinaryP transmission time of 1 kB payloads."""
    scn = scenarios.hotspot(n_senders=8, n_replicas=90, msg_num=30, payload_bytes=1000,
                            bandwidth_bytes_per_s=2_000_000)
    _compare(scn, engine_mod, oracle_mod)


@pytest.mark.one_geometry
def test_ping_pong_benched_shape_compact(engine_mod, oracle_mod):
    """bench.py's C2 per-replica shape -- 1,000 round trips
    (examples/ping-pong/Main.hs:53-79) on the compact geometry with forked
    children in place -- over 2,048 replicas, every field and node hash
    against the oracle's canonical order."""
    scn = scenarios.ping_pong(n_replicas=2048, round_trips=1000)
    with engine_mod.Engine(0) as e:
        e.load(scn, geometry="compact")
        assert e.geometry() == "compact"
        e.reset()
        st = e.run()
        res, hashes = e.results(), e.hashes()
    ores, ohashes = oracle_mod.run_batch(scn, threads=8)
    for f in FIELDS:
        assert np.array_equal(res[f], ores[f]), f
    assert np.array_equal(hashes, ohashes)
    assert st.events == int(ores["events"].sum()) > 2048 * 4000
