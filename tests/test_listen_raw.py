"""listenR (MonadDialog.hs:226-256) lowered host-side: the raw listener runs in
the handler's thread for every message reaching the port -- also for names
without a typed listener (:240-244) -- and the typed listener runs only when it
returned True (:246-253).  Checked on the oracle with counts derived from the
scenario (the gatekeeper server accepts even payloads).  CPU only; the GPU
parity case is in tests/test_gpu_parity.py."""
import numpy as np
import pytest

from timewarp import isa, scenarios
from timewarp.program import Program


@pytest.mark.parametrize("clients,msgs,junk", [(3, 8, 4), (5, 20, 3)])
def test_raw_listener_gates_typed_listener(oracle_mod, clients, msgs, junk):
    raw = scenarios.gatekeeper(n_clients=clients, n_replicas=4, msg_num=msgs, junk_every=junk)
    plain = scenarios.gatekeeper(n_clients=clients, n_replicas=4, msg_num=msgs, junk_every=junk, raw=False)
    rr, _ = oracle_mod.run_batch(raw, threads=4)
    rp, _ = oracle_mod.run_batch(plain, threads=4)
    assert (rr["status"] == 1).all() and (rp["status"] == 1).all()
    reqs = clients * msgs
    payloads = np.arange(reqs)
    junks = int((payloads % junk == junk - 1).sum())  # a Junk follows every Req whose payload is -1 mod junk_every
    acks_raw = int((payloads % 2 == 0).sum())
    # listenR: every Req and Junk reaches a handler thread; Acks only for accepted Reqs
    assert (rr["delivered"] == reqs + junks + acks_raw).all()
    assert (rr["undeliverable"] == 0).all()
    # plain listen (= listenR with `const $ return True`, :216-219): every Req
    # is answered; Junk has no typed listener but still reaches a thread
    assert (rp["delivered"] == 2 * reqs + junks).all()
    assert (rp["undeliverable"] == 0).all()
    assert (rr["dropped"] == 0).all() and (rp["dropped"] == 0).all()


def test_raw_listener_table_covers_every_kind():
    p = Program()
    seen = []

    def raw(c, accept):
        seen.append(accept)
        c.jmp(accept)

    s = p.listener_set({"A": "ha"}, raw=raw)
    plain = p.listener_set({"A": "ha"})
    p.kind("B")
    p.function("ha").end()
    img = p.finalize()
    assert len(seen) == 2  # one expansion per message kind
    for k in (p.kind("A"), p.kind("B")):
        assert img.listener_pc[s, k] != isa.PC_NONE
    # a plain listen's unknown name ends in a shared "no listener" stub
    assert img.listener_pc[plain, p.kind("B")] != isa.PC_NONE
    assert img.listener_pc[plain, p.kind("B")] != img.listener_pc[plain, p.kind("A")]
    assert img.listener_pc[s, p.kind("A")] != img.listener_pc[plain, p.kind("A")]


def test_raw_listener_accepting_everything_matches_listen_for_typed_names(oracle_mod):
    """`listenH = listenR ... (const $ return True)` (MonadDialog.hs:216-219):
    with an always-True raw listener and no foreign names, the outcome equals
    a plain listen: same clock, pops and message counts (node hashes differ,
    since pop terms carry the resumed pc and the raw entry moves it)."""
    def build(raw):
        p = Program()
        K = p.kind("M")
        s = p.listener_set({"M": "on_m"}, raw=raw)
        c = p.function("main")
        c.listen(s)
        c.seti(0, 5).link(1, 0)
        for _ in range(3):
            c.send(1, K, 0).wait(scenarios.for_(10))
        c.unlisten().end()
        c = p.function("on_m")
        c.trace(scenarios.TAG_REQ, 0).end()
        return p.finalize()
    from timewarp.scenario import Scenario, Topology
    outs = []
    for raw in (None, lambda c, acc: c.jmp(acc)):
        img = build(raw)
        topo = Topology.from_out_lists(1, [[0]])
        table = np.full((1, 1, 1), 7, np.uint32)
        scn = Scenario(name="loop", image=img, topo=topo, n_replicas=1, main_pc=img.pc_of("main"),
                       main_node=0, link_table=table, max_slots=32, queue_capacity=128)
        r, h = oracle_mod.run_batch(scn, threads=1)
        outs.append((r, h))
    (r0, h0), (r1, h1) = outs
    for k in ("final_t", "events", "delivered", "undeliverable", "status"):
        assert np.array_equal(r0[k], r1[k]), k
    assert int(r0["delivered"][0]) == 3
