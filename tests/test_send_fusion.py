"""SEND fused with its LINK / RLINK (include/timewarp.h TW_SEND_VIA_*,
Program.finalize's peephole): the fused image must run exactly as the unfused
one -- same pcs, yields, events and trace hashes; only the instruction count
per step shrinks.  CPU tests pin the peephole and the oracle's fused SEND;
GPU tests run fused and unfused images through the event, LP and batched-LP
kernels and require bit-equal results."""
import numpy as np
import pytest

from timewarp import isa, scenarios
from timewarp.abi import RESULT_FIELDS
from timewarp.program import Program
from timewarp.scenario import Scenario, Topology

SCENARIOS = {
    "hotspot": lambda: scenarios.hotspot(n_senders=8, n_replicas=4, msg_num=30),
    "hotspot_inline": lambda: scenarios.hotspot(n_senders=8, n_replicas=4, msg_num=30, fork_strategy="inline"),
    "gossip": lambda: scenarios.gossip(300, seed=7, drop_log2=3),
    "ping_pong": lambda: scenarios.ping_pong(n_replicas=4, round_trips=5),
    "token_ring": lambda: scenarios.token_ring(n_nodes=8, n_replicas=2, launch_duration=2_000_000),
    "gatekeeper": lambda: scenarios.gatekeeper(n_clients=4, n_replicas=2, msg_num=10),
}


def _pair(name, monkeypatch):
    fused = SCENARIOS[name]()
    monkeypatch.setenv("TW_FUSE_SEND", "0")
    plain = SCENARIOS[name]()
    monkeypatch.delenv("TW_FUSE_SEND")
    return fused, plain


def _n_fused(img):
    w = img.insns[:, 0].astype(np.int64)
    return int((((w & 0xFF) == isa.OP_SEND) & (((w >> 16) & (isa.SEND_VIA_LINK | isa.SEND_VIA_RLINK)) != 0)).sum())


def _send_prog(payload_reg=0, jump_to_send=False, rlink_from=None):
    """main on node 0: LINK/RLINK r1 ; SEND r1 over node 0's self-link, to its
    own listener, which traces the payload; optionally a second path jumps
    straight to the pair's SEND."""
    p = Program()
    s = p.listener_set({"M": "h"})
    c = p.function("main")
    c.listen(s).seti(0, 7).seti(2, 0)
    if jump_to_send:
        c.link(1, 0)
    if rlink_from is not None:
        c.seti(2, rlink_from).reply_link(1, 2)
    else:
        c.link(1, 0)
    pair_send = p.label("pair_send")
    p.bind(pair_send)
    c.send(1, "M", payload_reg)
    if jump_to_send:
        c.addi(2, 1).jnei(2, 2, pair_send)
    c.end()
    h = p.function("h")
    h.trace(5, 0).end()
    img = p.finalize()
    topo = Topology.from_out_lists(1, [[0]])
    return Scenario(name="send_pair", image=img, topo=topo, n_replicas=1, main_pc=img.pc_of("main"), main_node=0,
                    max_slots=16, queue_capacity=64, run_capacity=16, max_timeouts=4)


# ---------------------------------------------------------------- CPU


@pytest.mark.parametrize("name", sorted(SCENARIOS))
def test_oracle_fused_equals_unfused(oracle_mod, monkeypatch, name):
    fused, plain = _pair(name, monkeypatch)
    assert _n_fused(fused.image) > 0 and _n_fused(plain.image) == 0
    # the pair's second slot is kept: same length, same labels
    assert len(fused.image.insns) == len(plain.image.insns)
    rf, hf = oracle_mod.run_batch(fused, threads=2)
    rp, hp = oracle_mod.run_batch(plain, threads=2)
    for f in RESULT_FIELDS:
        assert np.array_equal(rf[f], rp[f]), f
    assert np.array_equal(hf, hp)


def test_peephole_shapes(monkeypatch):
    img = _send_prog().image
    assert _n_fused(img) == 1
    # payload register = the link register: the pair stays unfused
    assert _n_fused(_send_prog(payload_reg=1).image) == 0
    r = _send_prog(rlink_from=0).image
    w = r.insns[:, 0].astype(np.int64)
    k = np.nonzero(((w & 0xFF) == isa.OP_SEND) & (((w >> 16) & isa.SEND_VIA_RLINK) != 0))[0]
    assert k.size == 1 and ((int(w[k[0]]) >> 28) & 3) == 2 and int(r.insns[k[0], 1]) == 0


@pytest.mark.parametrize("kw", [{}, {"payload_reg": 1}, {"jump_to_send": True}, {"rlink_from": 0}, {"rlink_from": 99}])
def test_oracle_pair_programs(oracle_mod, monkeypatch, kw):
    """A jump into the pair's SEND sends over r1 as before; an out-of-range
    reply link stops the replica in both images."""
    fused = _send_prog(**kw)
    monkeypatch.setenv("TW_FUSE_SEND", "0")
    plain = _send_prog(**kw)
    rf, hf = oracle_mod.run_batch(fused, threads=1)
    rp, hp = oracle_mod.run_batch(plain, threads=1)
    for f in RESULT_FIELDS:
        assert np.array_equal(rf[f], rp[f]), f
    assert np.array_equal(hf, hp)
    if kw.get("rlink_from") == 99:
        assert int(rf["status"][0]) == isa.REP_ERR_INSN
    else:
        assert int(rf["status"][0]) == isa.REP_DONE and int(rf["delivered"][0]) >= 1


# ---------------------------------------------------------------- GPU


def _gpu_run(engine_mod, scn, geometry=None):
    with engine_mod.Engine(0) as e:
        e.load(scn, geometry=geometry)
        e.reset()
        e.run()
        return e.results(), e.hashes()


@pytest.mark.gpu
@pytest.mark.one_geometry
@pytest.mark.parametrize("name", sorted(SCENARIOS))
@pytest.mark.parametrize("geometry", [None, "wave", "lpb"])
def test_gpu_fused_equals_unfused(engine_mod, oracle_mod, monkeypatch, name, geometry):
    fused, plain = _pair(name, monkeypatch)
    try:
        rf, hf = _gpu_run(engine_mod, fused, geometry)
    except engine_mod.EngineError:
        if geometry == "lpb" and name == "gatekeeper":
            pytest.skip("gatekeeper's raw listener reads another node's state: not a batched-LP scenario")
        raise
    rp, hp = _gpu_run(engine_mod, plain, geometry)
    ro, ho = oracle_mod.run_batch(fused, threads=4)
    for f in RESULT_FIELDS:
        if f == "tie_flags":
            continue
        assert np.array_equal(rf[f], rp[f]), (f, rf[f][:4], rp[f][:4])
        assert np.array_equal(rf[f], ro[f]), (f, rf[f][:4], ro[f][:4])
    assert np.array_equal(hf, hp) and np.array_equal(hf, ho)


@pytest.mark.gpu
@pytest.mark.one_geometry
@pytest.mark.parametrize("kw", [{}, {"jump_to_send": True}, {"rlink_from": 0}, {"rlink_from": 99}])
def test_gpu_pair_programs(engine_mod, oracle_mod, kw):
    scn = _send_prog(**kw)
    rf, hf = _gpu_run(engine_mod, scn)
    ro, ho = oracle_mod.run_batch(scn, threads=1)
    for f in RESULT_FIELDS:
        if f == "tie_flags":
            continue
        assert np.array_equal(rf[f], ro[f]), f
    assert np.array_equal(hf, ho)


@pytest.mark.gpu
@pytest.mark.one_geometry
@pytest.mark.parametrize("parts", [1, 3])
def test_gpu_partitioned_fused_equals_unfused(engine_mod, monkeypatch, parts):
    """Node-partitioned LP mode (config 4's engine): the lane's cached out-link
    base and reply link serve the fused halves."""
    fused, plain = _pair("gossip", monkeypatch)
    af, hf, _ = engine_mod.run_partitioned(fused, parts=parts)
    ap, hp, _ = engine_mod.run_partitioned(plain, parts=parts)
    for f in ("final_t", "events", "delivered", "dropped", "undeliverable", "status", "main_exc", "threads"):
        assert int(af[f]) == int(ap[f]), f
    assert np.array_equal(hf, hp)
