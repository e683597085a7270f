"""Fused instruction pairs (Program.finalize's peephole, include/timewarp.h):
SEND with its LINK / RLINK (TW_SEND_VIA_*), an ALU op with the NSTORE of its
result (TW_ALU_NSTORE) and two TRACEs (TW_TRACE_PAIR).  The fused image must
run exactly as the unfused one -- same pcs, yields, events and trace hashes;
only the instruction count per step shrinks.  CPU tests pin the peephole and the oracle's fused SEND;
GPU tests run fused and unfused images through the event, LP and batched-LP
kernels and require bit-equal results."""
import numpy as np
import pytest

from timewarp import isa, scenarios
from timewarp.abi import RESULT_FIELDS
from timewarp.program import Program
from timewarp.scenario import Scenario, Topology
from timewarp.timeunits import for_

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
    monkeypatch.setenv("TW_FUSE_PAIRS", "0")
    plain = SCENARIOS[name]()
    monkeypatch.delenv("TW_FUSE_PAIRS")
    return fused, plain


def _n_fused(img):
    w = img.insns[:, 0].astype(np.int64)
    return int((((w & 0xFF) == isa.OP_SEND) & (((w >> 16) & (isa.SEND_VIA_LINK | isa.SEND_VIA_RLINK)) != 0)).sum())


def _n_flag(img, ops, flag=0x8000):
    w = img.insns[:, 0].astype(np.int64)
    return int((np.isin(w & 0xFF, ops) & (((w >> 16) & flag) != 0)).sum())


def _pair_prog(jump_into=False, n_traces=3):
    """main: SETI/NOW/ADDI results stored to node vars through fused pairs, a
    run of TRACEs (overlapping pairs), optionally a second lap that jumps to
    the pairs' second instructions; the node vars are traced at the end."""
    p = Program()
    c = p.function("main")
    c.seti(3, 0)
    top = c.here()
    c.seti(0, 41)
    nst = p.label("nst")
    p.bind(nst)
    c.nstore(0, 0)
    c.now(1).nstore(1, 1).addi(0, 1).nstore(0, 2)
    c.wait(for_(1000))
    tr2 = p.label("tr2")
    c.trace(11, 0)
    p.bind(tr2)
    for k in range(1, n_traces):
        c.trace(11 + k, k % 4)
    c.nload(2, 0).trace(20, 2).nload(2, 1).trace(21, 2).nload(2, 2).trace(22, 2)
    if jump_into:
        c.addi(3, 1).jeqi(3, 2, "done").jeqi(3, 1, "second")
        c.jmp(top)
        c2 = p.function("second")
        c2.seti(0, 7).jmp(nst)
        p.bind(p.label("done"))
    c.end()
    img = p.finalize()
    topo = Topology.from_out_lists(1, [[]])
    return Scenario(name="pairs", image=img, topo=topo, n_replicas=3, main_pc=img.pc_of("main"), main_node=0,
                    max_slots=8, queue_capacity=32, run_capacity=8, max_timeouts=2)


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


def test_peephole_alu_and_trace_pairs(monkeypatch):
    img = _pair_prog().image
    assert _n_flag(img, [isa.OP_SETI, isa.OP_NOW, isa.OP_ADDI]) == 3
    assert _n_flag(img, [isa.OP_TRACE]) == 2  # 3 TRACEs in a row: two overlapping pairs
    monkeypatch.setenv("TW_FUSE_PAIRS", "0")
    assert _n_flag(_pair_prog().image, [isa.OP_SETI, isa.OP_NOW, isa.OP_ADDI, isa.OP_TRACE]) == 0


@pytest.mark.parametrize("kw", [{}, {"jump_into": True}, {"n_traces": 2}, {"n_traces": 5, "jump_into": True}])
def test_oracle_alu_trace_pairs(oracle_mod, monkeypatch, kw):
    fused = _pair_prog(**kw)
    monkeypatch.setenv("TW_FUSE_PAIRS", "0")
    plain = _pair_prog(**kw)
    rf, hf = oracle_mod.run_batch(fused, threads=1)
    rp, hp = oracle_mod.run_batch(plain, threads=1)
    for f in RESULT_FIELDS:
        assert np.array_equal(rf[f], rp[f]), f
    assert np.array_equal(hf, hp)
    assert (rf["status"] == isa.REP_DONE).all()


@pytest.mark.parametrize("kw", [{}, {"payload_reg": 1}, {"jump_to_send": True}, {"rlink_from": 0}, {"rlink_from": 99}])
def test_oracle_pair_programs(oracle_mod, monkeypatch, kw):
    """A jump into the pair's SEND sends over r1 as before; an out-of-range
    reply link stops the replica in both images."""
    fused = _send_prog(**kw)
    monkeypatch.setenv("TW_FUSE_PAIRS", "0")
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
@pytest.mark.parametrize("geometry", [None, "dense", "sparse", "wave", "narrow", "compact"])
@pytest.mark.parametrize("kw", [{}, {"jump_into": True}, {"n_traces": 5, "jump_into": True}])
def test_gpu_alu_trace_pairs(engine_mod, oracle_mod, kw, geometry):
    scn = _pair_prog(**kw)
    rf, hf = _gpu_run(engine_mod, scn, geometry)
    ro, ho = oracle_mod.run_batch(scn, threads=1)
    for f in RESULT_FIELDS:
        if f == "tie_flags":
            continue
        assert np.array_equal(rf[f], ro[f]), (f, rf[f], ro[f])
    assert np.array_equal(hf, ho)


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
