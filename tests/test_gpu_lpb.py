"""Batched node-partitioned mode (tw_lpb_load) vs the oracle (canonical mode).

Every (node, replica) pair is a logical process; the replicas share one
device-driven window loop.  The sequential TimedT run of each replica
(oracle/timedt_oracle.cpp, TimedT.hs:234-304) must come out bit-exact: every
result field and every per-node trace hash.  Main's forks onto the node
daemons travel as spawn records; a hotspot receiver with more than TW_LIGHT
records pending takes the tw_lp_due path (its due run, sorted per window)."""
import numpy as np
import pytest

from timewarp import scenarios
from timewarp.abi import RESULT_FIELDS

pytestmark = [pytest.mark.gpu, pytest.mark.one_geometry]


def _compare_lpb(scn, engine_mod, oracle_mod, threads=8):
    with engine_mod.Engine(0) as e:
        e.load(scn, geometry="lpb")
        assert e.geometry() == "lpb"
        e.reset()
        st = e.run()
        res, hashes = e.results(), e.hashes()
        windows, ticks = e.lpb_windows()
    ores, ohashes = oracle_mod.run_batch(scn, threads=threads)
    bad = {}
    for f in RESULT_FIELDS:
        if f == "tie_flags":
            continue
        m = np.nonzero(res[f] != ores[f])[0]
        if m.size:
            bad[f] = (m[:5].tolist(), res[f][m[:5]].tolist(), ores[f][m[:5]].tolist())
    hm = np.nonzero((hashes != ohashes).any(axis=1))[0]
    if hm.size:
        bad["hashes"] = (hm[:5].tolist(), np.nonzero(hashes[hm[0]] != ohashes[hm[0]])[0][:8].tolist())
    assert not bad, f"{scn.name}: LPB != oracle: {bad}"
    assert st.events == int(ores["events"].sum())
    assert windows > 0 and ticks >= windows
    return st, ores, windows


def test_lpb_hotspot_light(engine_mod, oracle_mod):
    # 8 senders: the receiver's inbox stays light (<= 32 pending)
    scn = scenarios.hotspot(n_senders=8, n_replicas=64, msg_num=30)
    _compare_lpb(scn, engine_mod, oracle_mod)


def test_lpb_hotspot_heavy_receiver(engine_mod, oracle_mod):
    # 64 senders at 1 msg/ms with 1-5 ms delays: ~300 pings pending at the
    # receiver, so its records go through tw_lp_due every window
    scn = scenarios.hotspot(n_senders=64, n_replicas=32, msg_num=60)
    st, ores, windows = _compare_lpb(scn, engine_mod, oracle_mod)
    assert ores["delivered"].sum() == 2 * 64 * 60 * 32


def test_lpb_hotspot_inline(engine_mod, oracle_mod):
    # ForkStrategy `const id`: the handler runs in the phantom deliverer
    scn = scenarios.hotspot(n_senders=48, n_replicas=16, msg_num=40, fork_strategy="inline")
    _compare_lpb(scn, engine_mod, oracle_mod)


def test_lpb_hotspot_full_senders(engine_mod, oracle_mod):
    # the C5 shape (256 senders), few replicas and messages
    scn = scenarios.hotspot(n_senders=256, n_replicas=4, msg_num=12)
    _compare_lpb(scn, engine_mod, oracle_mod)


def test_lpb_ping_pong(engine_mod, oracle_mod):
    scn = scenarios.ping_pong(n_replicas=256, round_trips=30)
    _compare_lpb(scn, engine_mod, oracle_mod)


def test_lpb_gossip_single_replica(engine_mod, oracle_mod):
    # one replica: the classic partitioned scenario through the batched path
    scn = scenarios.gossip(n_nodes=4096, fanout=4)
    _compare_lpb(scn, engine_mod, oracle_mod, threads=1)


def test_lpb_token_ring_two_phase(engine_mod, oracle_mod):
    # the observer is fed by 0 µs links: it runs in phase 1 of every window,
    # after the ring nodes; main's forks onto every node are spawn records
    scn = scenarios.token_ring(n_nodes=16, n_replicas=64, launch_duration=40_000_000, drop_log2=3)
    st, ores, windows = _compare_lpb(scn, engine_mod, oracle_mod)
    assert ores["dropped"].sum() > 0 and ores["delivered"].sum() > 0


def test_lpb_token_ring_many_nodes(engine_mod, oracle_mod):
    # C3's node count (spawns over several windows, the teardown burst at
    # launchDuration), few replicas
    scn = scenarios.token_ring(n_nodes=4096, n_replicas=4, launch_duration=20_000_000, drop_log2=10)
    _compare_lpb(scn, engine_mod, oracle_mod)


def test_lpb_token_ring_c3_per_gpu_shape(engine_mod, oracle_mod):
    # the path bench.py takes for C3 at <= 8,192 replicas per GPU (BASELINE's
    # 64k over 8 GPUs) at its real shape: 4,096 nodes, launchDuration 120 s
    # (start-up fork chain, ~40 token hops, the teardown kills), drop 2^-10
    scn = scenarios.token_ring(n_nodes=4096, n_replicas=4, launch_duration=120_000_000, drop_log2=10)
    st, ores, windows = _compare_lpb(scn, engine_mod, oracle_mod)
    assert (ores["status"] == 1).all() and ores["delivered"].sum() > 0


def test_lpb_token_ring_c3_per_gpu_shape_64(engine_mod, oracle_mod):
    # the same shape over 64 replicas (lanes = node << 6 | replica: waves of 64
    # replicas of one node, as at 8,192 replicas per GPU)
    scn = scenarios.token_ring(n_nodes=4096, n_replicas=64, launch_duration=120_000_000, drop_log2=10)
    _compare_lpb(scn, engine_mod, oracle_mod)


def test_lpb_rejects_short_link_out_of_phase1(engine_mod):
    # a link shorter than the lookahead out of a node that itself is fed by one
    # would need a third phase: tw_lpb_load refuses it
    scn = scenarios.gossip(n_nodes=64, fanout=2)
    lt = scn.link_table.copy()
    a = 0
    l_ab = int(scn.topo.out_off[a])
    b = int(scn.topo.dst[l_ab])
    l_bc = int(scn.topo.out_off[b])
    lt[l_ab] = 0
    lt[l_bc] = 0
    scn.link_table = lt
    with engine_mod.Engine(0) as e:
        with pytest.raises(engine_mod.EngineError):
            e.load_lpb(scn, lookahead_us=1000)


def test_lpb_equals_replica_kernel_at_scale(engine_mod):
    # GPU vs GPU at a size the oracle would take minutes for: the C5 shape with
    # 64 replicas and 200 messages per sender, batched logical processes vs the
    # wavefront-per-replica kernel (itself oracle-checked), every output field
    # and node hash
    scn = scenarios.hotspot(n_senders=256, n_replicas=64, msg_num=200)
    with engine_mod.Engine(0) as e:
        e.load(scn, geometry="lpb")
        e.reset()
        e.run()
        r1, h1 = e.results(), e.hashes()
    with engine_mod.Engine(0) as e:
        e.load(scn, geometry="wave")
        e.run()
        r2, h2 = e.results(), e.hashes()
    for f in RESULT_FIELDS:
        if f != "tie_flags":
            assert np.array_equal(r1[f], r2[f]), f
    assert np.array_equal(h1, h2)
    assert (r1["status"] == 1).all() and r1["delivered"].sum() == 2 * 256 * 200 * 64


def test_lpb_hotspot_bandwidth(engine_mod, oracle_mod):
    # BinaryP wire sizes -> transmission time added to each link delay
    # (Message.hs:155-202): the lookahead is the smallest delay including it
    scn = scenarios.hotspot(n_senders=32, n_replicas=16, msg_num=40, payload_bytes=512,
                            bandwidth_bytes_per_s=2_000_000)
    _compare_lpb(scn, engine_mod, oracle_mod)


def test_lpb_token_ring_laps(engine_mod, oracle_mod):
    # the token goes round the ring twice (every ring node's worker woken by a
    # throwTo from its server's handler, notes to the phase-1 observer each hop)
    N = 12
    scn = scenarios.token_ring(n_nodes=N, n_replicas=32, launch_duration=(2 * N + 2) * 3_000_000 + 5_000_000,
                               drop_log2=6)
    st, ores, windows = _compare_lpb(scn, engine_mod, oracle_mod)
    assert ores["delivered"].sum() > 2 * 2 * N * 32 * 0.5


@pytest.mark.parametrize("bad", ["replicas", "inbox"])
def test_lpb_load_validation(engine_mod, bad):
    # the replica count must be a power of two (lanes are node << log2 R |
    # replica) and a node's inbox at most 2048 records (tw_lp_due stages it in LDS)
    if bad == "replicas":
        scn = scenarios.hotspot(n_senders=4, n_replicas=12, msg_num=4)
        cap = None
    else:
        scn = scenarios.hotspot(n_senders=4, n_replicas=8, msg_num=4)
        cap = np.full(scn.n_nodes, 4096, np.uint32)
    with engine_mod.Engine(0) as e:
        with pytest.raises(engine_mod.EngineError):
            e.load_lpb(scn, node_inbox_cap=cap)


@pytest.mark.parametrize("recv_cap", [2, 48])
def test_lpb_inbox_overflow_is_an_error(engine_mod, oracle_mod, recv_cap):
    # an undersized receiver inbox: 2 records (light path: the drain clamps the
    # overflowed count to the capacity) or 48 of the ~300 pending (heavy path:
    # tw_lp_due); the run must stop with TW_ERR_REPLICA, not read past the
    # lane's records, and the device stays usable for a correct run after it
    S = 64
    scn = scenarios.hotspot(n_senders=S, n_replicas=16, msg_num=40)
    caps = np.array(scn.meta["lp_inbox_cap"], np.uint32)
    assert caps[S] > recv_cap
    bad = caps.copy()
    bad[S] = recv_cap
    with engine_mod.Engine(0) as e:
        e.load_lpb(scn, node_inbox_cap=bad)
        e.reset()
        with pytest.raises(engine_mod.EngineError, match=r"failed: -6 "):
            e.run()
    _compare_lpb(scn, engine_mod, oracle_mod)


@pytest.mark.parametrize("windows", ["per_replica", "global"])
@pytest.mark.parametrize("case", ["token_ring_two_phase", "token_ring_many_nodes", "hotspot_heavy", "gossip"])
def test_lpb_grid_stride_work_list(engine_mod, oracle_mod, monkeypatch, case, windows):
    """Contexts of more than TW_LP_GRID workgroups of lanes (C3's 33.6M lanes
    at 8,192 replicas) launch TW_LP_GRID workgroups that walk the window's
    work list grid-stride; a grid of 3 workgroups makes every list take many
    passes.  Both window modes: every replica in its own window (the default)
    and one window for the whole batch (TW_LPB_GLOBAL=1, where the work-list
    scan skips idle 256-lane blocks)."""
    monkeypatch.setenv("TW_LP_GRID", "3")
    if windows == "global":
        monkeypatch.setenv("TW_LPB_GLOBAL", "1")
    scn = {
        "token_ring_two_phase": lambda: scenarios.token_ring(n_nodes=16, n_replicas=64, launch_duration=40_000_000,
                                                             drop_log2=3),
        "token_ring_many_nodes": lambda: scenarios.token_ring(n_nodes=4096, n_replicas=4, launch_duration=20_000_000,
                                                              drop_log2=10),
        "hotspot_heavy": lambda: scenarios.hotspot(n_senders=64, n_replicas=32, msg_num=60),
        "gossip": lambda: scenarios.gossip(n_nodes=4096, fanout=4),
    }[case]()
    _compare_lpb(scn, engine_mod, oracle_mod, threads=1 if case == "gossip" else 8)


@pytest.mark.parametrize("case", ["token_ring_drift", "hotspot"])
def test_lpb_per_replica_windows_fewer(engine_mod, oracle_mod, monkeypatch, case):
    """Per-replica windows: the replicas' token hops drift apart, so one
    window for the whole batch has to cover the union of their event times;
    every replica in its own window takes fewer windows for the same,
    bit-exact outputs."""
    scn = {
        "token_ring_drift": lambda: scenarios.token_ring(n_nodes=32, n_replicas=64, launch_duration=30_000_000,
                                                         drop_log2=6),
        "hotspot": lambda: scenarios.hotspot(n_senders=16, n_replicas=32, msg_num=40),
    }[case]()
    _, _, w_rep = _compare_lpb(scn, engine_mod, oracle_mod)
    monkeypatch.setenv("TW_LPB_GLOBAL", "1")
    _, _, w_glob = _compare_lpb(scn, engine_mod, oracle_mod)
    assert w_rep <= w_glob, (w_rep, w_glob)
    if case == "token_ring_drift":
        assert w_rep < w_glob, (w_rep, w_glob)


# ---- batched delivery (tw_lp_due runs a heavy receiver's due run data-parallel)

def _lpb_batched(scn, engine_mod, oracle_mod, threads=8):
    """The run vs the oracle, plus (batched, due) of tw_lpb_batch."""
    with engine_mod.Engine(0) as e:
        e.load(scn, geometry="lpb")
        e.reset()
        st = e.run()
        res, hashes = e.results(), e.hashes()
        bat = e.lpb_batch()
    ores, ohashes = oracle_mod.run_batch(scn, threads=threads)
    for f in RESULT_FIELDS:
        if f != "tie_flags":
            assert np.array_equal(res[f], ores[f]), (scn.name, f)
    assert np.array_equal(hashes, ohashes), scn.name
    assert st.events == int(ores["events"].sum())
    return ores, bat


def test_lpb_batched_delivery_heavy_receiver(engine_mod, oracle_mod):
    """bench/Network's Ping handler (Receiver/Main.hs:32-38) is batchable: most
    of the receiver's due records run one per thread in tw_lp_due, and every
    field and node hash still equals the sequential oracle."""
    scn = scenarios.hotspot(n_senders=64, n_replicas=32, msg_num=60)
    ores, (bat, due) = _lpb_batched(scn, engine_mod, oracle_mod)
    assert due > 0 and bat >= 0.5 * due, (bat, due)


def test_lpb_batched_delivery_off_is_the_chain(engine_mod, oracle_mod, monkeypatch):
    """TW_LP_BATCH=0: every due record on the receiver's chain; same results."""
    monkeypatch.setenv("TW_LP_BATCH", "0")
    scn = scenarios.hotspot(n_senders=64, n_replicas=32, msg_num=60)
    ores, (bat, due) = _lpb_batched(scn, engine_mod, oracle_mod)
    assert bat == 0 and due > 0


def test_lpb_batched_delivery_refuses_a_stateful_handler(engine_mod, oracle_mod):
    """A Ping handler that counts its pings in a node variable (NSTORE) is not
    batchable (classify_batch): the due run stays on the chain."""
    scn = scenarios.hotspot(n_senders=64, n_replicas=16, msg_num=40, receiver_counter=True)
    ores, (bat, due) = _lpb_batched(scn, engine_mod, oracle_mod)
    assert bat == 0 and due > 0


def test_lpb_batched_delivery_drops_and_undeliverable(engine_mod, oracle_mod):
    """Dropped pongs (DROP terms, no resume) and pings that reach the receiver
    after its `unlisten` at 1 s (undeliverable: the stopper ran first, so the
    prefix before it and the records after it both batch)."""
    scn = scenarios.hotspot(n_senders=64, n_replicas=16, msg_num=2000, duration_s=1, drop_log2=2)
    ores, (bat, due) = _lpb_batched(scn, engine_mod, oracle_mod)
    assert ores["dropped"].sum() > 0 and ores["undeliverable"].sum() > 0
    assert bat > 0


def test_lpb_batched_delivery_c5_shape(engine_mod, oracle_mod):
    """The C5 receiver: 256 senders, ~256 pings per 1-ms window."""
    scn = scenarios.hotspot(n_senders=256, n_replicas=16, msg_num=100)
    ores, (bat, due) = _lpb_batched(scn, engine_mod, oracle_mod)
    assert bat >= 0.5 * due


def test_lpb_batched_delivery_benched_shape_256(engine_mod, oracle_mod):
    """C5's full message count on a 256-replica batch: 256 senders x 1,000
    messages each, every replica against the sequential oracle (the bench's
    own check samples ~1k of 4,096 replicas; tools/parity_all.py runs all)."""
    scn = scenarios.hotspot(n_senders=256, n_replicas=256, msg_num=1000)
    ores, (bat, due) = _lpb_batched(scn, engine_mod, oracle_mod, threads=16)
    assert ores["delivered"].sum() == 2 * 256 * 1000 * 256
    assert bat >= 0.5 * due, (bat, due)


def test_lpb_batched_delivery_over_the_cap(engine_mod, oracle_mod):
    """More than TW_BATCH_CAP (1,024) due records per lane and window: one
    sender pinging every 3 µs (a 2-µs wait and the send's 1-µs yield) over
    4-ms links puts ~1,333 pings in each 4-ms window's due run (and as many
    pongs in the sender's), 3 µs apart, so every record's handler has ended
    before the next one's wake: the batch takes exactly the cap -- the prefix
    closed by the first record past it -- and the rest runs on
    the chain, bit-exact against the oracle."""
    scn = scenarios.hotspot(n_senders=1, n_replicas=8, msg_num=4000, msg_rate=500_000, duration_s=1,
                            network_delay=(4000, 4000))
    # (both ends heavy: ~1,333 records in flight each way; a tick's outbox
    # holds them all)
    scn.meta = dict(scn.meta, lp_outbox_cap=1 << 16, lp_inbox_cap=np.array([2048, 2048, 4], np.uint32))
    ores, (bat, due) = _lpb_batched(scn, engine_mod, oracle_mod)
    assert due > 2 * 1024 and bat >= 1024, (bat, due)


def test_lpb_batched_delivery_full_lane_fails_like_the_chain(engine_mod, oracle_mod, monkeypatch):
    """A lane with no free thread slot: on the chain the first due pop fails
    the replica with TW_REP_ERR_SLOTS (alloc_slot), so the batch must leave
    such a lane's due run to the chain.  One slot per lane: every
    node's own thread fills it, nothing is batched, and the batched and the
    chain runs end the same, field for field and hash for hash.  (A replica
    error is a status, not a tw_run failure; and after a capacity failure a
    logical process's counts are its own, not the sequential oracle's, whose
    thread cap is the replica's.)"""
    import copy

    base = scenarios.hotspot(n_senders=64, n_replicas=16, msg_num=40)
    scn = copy.copy(base)
    scn.meta = dict(base.meta, lp_max_slots=1)
    out = {}
    for mode in ("1", "0"):
        monkeypatch.setenv("TW_LP_BATCH", mode)
        with engine_mod.Engine(0) as e:
            e.load(scn, geometry="lpb")
            e.reset()
            st = e.run()
            out[mode] = (e.results(), e.hashes(), e.lpb_batch(), st)
    (r1, h1, (b1, d1), s1), (r0, h0, (b0, _), _) = out["1"], out["0"]
    assert b1 == 0 and b0 == 0 and d1 > 0, (b1, b0, d1)
    assert (r1["status"] == 3).all() and s1.replicas_error == 16  # TW_REP_ERR_SLOTS
    for f in RESULT_FIELDS:
        if f != "tie_flags":
            assert np.array_equal(r1[f], r0[f]), f
    assert np.array_equal(h1, h0)
