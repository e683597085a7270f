"""ABI-2 semantics on the oracle (CPU): the unbounded handler stack, full-width
exception payloads, tie-order probes, `close` resetting a connection's state,
and BinaryP transmission time at send."""
import numpy as np
import pytest

import progs
from timewarp import isa, scenarios


def _cps(r):
    return [v for (_, _, k, v) in r.traces if k == progs.TAG_CP]


def test_deep_handler_stack_unwinds_level_by_level(oracle_mod):
    """Frames 0..7 = Arith, async, finally, async, Arith, finally, Arith, async.
    ThreadKilled lands in the innermost async frame (7); each handler rethrows
    Overflow, caught by the next Arith frame below: 6, 4, 0 (finally frames on
    the way set their done flag).  TimedT.hs:183-204 + ExceptionSpec.hs:219-229."""
    v = (1 << 40) + 7
    r = oracle_mod.run(progs.deep_catch_prog(8, max_frames=8, payload=v))
    assert r.result["status"] == isa.REP_DONE
    assert _cps(r) == [7, 6, 4, 0]
    assert [val for (_, _, k, val) in r.traces if k == progs.TAG_TS] == [v] * 4


def test_handler_stack_capacity_is_a_status(oracle_mod):
    r = oracle_mod.run(progs.deep_catch_prog(9, max_frames=8))
    assert r.result["status"] == isa.REP_ERR_FRAMES
    r = oracle_mod.run(progs.deep_catch_prog(3, max_frames=0))  # default: the record's two frames
    assert r.result["status"] == isa.REP_ERR_FRAMES


@pytest.mark.parametrize("v", [(1 << 40) + 3, -(1 << 50) - 1, (1 << 63) - 1])
def test_full_width_payload(oracle_mod, v):
    """`ValueReceived Int` (examples/token-ring/Main.hs:156) keeps all 64 bits."""
    r = oracle_mod.run(progs.payload_prog(v))
    assert [val for (_, _, k, val) in r.traces if k == progs.TAG_TS] == [v]


def test_tie_probes_flag_pqueue_divergence(oracle_mod):
    """The engine's tie probes (reverse / scrambled equal-timestamp order) flag a
    program only if its trace depends on the tie order; on the random programs
    they flag every program whose pqueue-mode trace differs at t_end=3000, and
    never one that pqueue agrees with."""
    def same(a, b):
        return a.result == b.result and np.array_equal(a.hashes, b.hashes)

    flagged = pq = 0
    for seed in range(40):
        s = progs.random_program(seed)
        r = [oracle_mod.run(s, mode=m, t_end=3000) for m in range(4)]
        probe = not same(r[0], r[2]) or not same(r[0], r[3])
        div = not same(r[0], r[1])
        assert probe == div, seed
        flagged += probe
        pq += div
    assert flagged == pq > 0


def test_tie_probes_leave_configs_unchanged(oracle_mod):
    """The BASELINE configs are tie-insensitive under the probes too."""
    for scn in (scenarios.token_ring(n_nodes=24, n_replicas=8, launch_duration=60_000_000, drop_log2=3,
                                     link_depth=8),
                scenarios.hotspot(n_senders=12, n_replicas=4, msg_num=30)):
        a, ha = oracle_mod.run_batch(scn, mode=0)
        for m in (oracle_mod.MODE_LIFO, oracle_mod.MODE_SCRAMBLE):
            b, hb = oracle_mod.run_batch(scn, mode=m)
            assert np.array_equal(a, b) and np.array_equal(ha, hb), (scn.name, m)


def test_close_resets_connection_state(oracle_mod):
    """socket-state with `close` every 2 pings: the per-connection request
    counter (userStateR) restarts at 1 on every new connection."""
    scn = scenarios.socket_state(n_replicas=8, close_every=2)
    for rep in range(8):
        r = oracle_mod.run(scn, rep)
        nos = [v for (_, _, k, v) in r.traces if k == scenarios.TAG_GOT_PING_NO]
        assert all(1 <= n <= 2 for n in nos), nos
    ref = scenarios.socket_state(n_replicas=8)
    counts = [max([v for (_, _, k, v) in oracle_mod.run(ref, i).traces if k == scenarios.TAG_GOT_PING_NO],
                  default=0) for i in range(8)]
    assert max(counts) > 2  # without close the counters keep growing


def test_binaryp_transmission_time(oracle_mod):
    """One ping-pong round trip: each message is delayed by its link delay plus
    ceil(bytes * 10^6 / bandwidth) µs (Message.hs:155-202 sizes)."""
    base = scenarios.ping_pong(n_replicas=1, round_trips=1)
    o0 = oracle_mod.run(base)
    s = scenarios.ping_pong(n_replicas=1, round_trips=1)
    s.msg_bytes = np.array([1000, 3000], np.uint32)        # Ping, Pong wire sizes
    s.link_bw = np.array([1_000_000, 2_000_000], np.uint64)  # ping->pong, pong->ping bytes/s
    o1 = oracle_mod.run(s)
    # Ping: 1000 B at 1 MB/s = 1000 µs; Pong: 3000 B at 2 MB/s = 1500 µs
    assert o1.result["final_t"] - o0.result["final_t"] == 1000 + 1500
