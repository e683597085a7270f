"""ForkStrategy (MonadDialog.hs:114-117,317) on the oracle: in-place dispatch
(`const id`) runs the listener in the delivering thread, so each delivered
message costs two pops fewer than with the default `fork_` (the forked
handler's start and the deliverer's resume after `wait (for 1 mcs)`), while
virtual time and message counts stay the same.  CPU only."""
import numpy as np
import pytest

from timewarp import isa, scenarios
from timewarp.program import Program


@pytest.mark.parametrize("senders,msgs", [(4, 10), (8, 40)])
def test_inline_saves_two_pops_per_delivery(oracle_mod, senders, msgs):
    f = scenarios.hotspot(n_senders=senders, n_replicas=3, msg_num=msgs)
    i = scenarios.hotspot(n_senders=senders, n_replicas=3, msg_num=msgs, fork_strategy="inline")
    rf, hf = oracle_mod.run_batch(f, threads=3)
    ri, hi = oracle_mod.run_batch(i, threads=3)
    assert (rf["status"] == 1).all() and (ri["status"] == 1).all()
    for k in ("final_t", "delivered", "dropped", "undeliverable"):
        assert np.array_equal(rf[k], ri[k]), k
    assert np.array_equal(rf["events"] - ri["events"], 2 * rf["delivered"])
    assert np.array_equal(rf["threads"] - ri["threads"], rf["delivered"])
    assert not np.array_equal(hf, hi)  # resume terms differ: the traces are not the same


def test_gossip_inline_same_outcome(oracle_mod):
    f = oracle_mod.run(scenarios.gossip(500, seed=3), trace_cap=0)
    i = oracle_mod.run(scenarios.gossip(500, seed=3, fork_strategy="inline"), trace_cap=0)
    for k in ("delivered", "dropped"):
        assert int(f.result[k]) == int(i.result[k]), k
    # the last pop of the forked run may be a deliverer's resume, 1 µs later
    assert 0 <= int(f.result["final_t"]) - int(i.result["final_t"]) <= 1
    assert int(f.result["events"]) - int(i.result["events"]) == 2 * int(f.result["delivered"])


def test_inline_flag_in_listener_table():
    p = Program()
    s0 = p.listener_set({"A": "ha", "B": "hb"}, inline=("B",))
    for name in ("ha", "hb"):
        p.function(name).end()
    img = p.finalize()
    ka, kb = p.kind("A"), p.kind("B")
    assert img.listener_pc[s0, ka] & isa.LPC_INLINE == 0
    assert img.listener_pc[s0, kb] & isa.LPC_INLINE
    with pytest.raises(ValueError):
        Program().listener_set({"A": "ha"}, inline=("C",))
    with pytest.raises(ValueError):
        scenarios.hotspot(n_senders=2, fork_strategy="sometimes")
