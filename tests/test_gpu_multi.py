"""Multi-device contexts behind the C ABI (tw_create(devices, ndev) and
tw_create_rank), on the one GPU of the test box:

  * several shards of one process: replicas split into contiguous blocks
    [g*R/G, (g+1)*R/G); a device listed several times makes
    the library move the LP record blocks and window words by device copies
    ordered with HIP events (the transport real multi-GPU contexts replace
    with RCCL);
  * a one-rank RCCL job (tw_comm_id + tw_create_rank): the statistics
    all-reduce, the record blocks (send/recv to itself), the window-word
    all-reduce(min) and the result / hash reductions go through the library's
    own RCCL communicator.

Every run must equal the oracle's sequential TimedT runs (TimedT.hs:234-304)
field by field and node hash by node hash, exactly like the single-device
engine."""
import numpy as np
import pytest

from timewarp import scenarios
from timewarp.abi import RESULT_FIELDS

pytestmark = [pytest.mark.gpu, pytest.mark.one_geometry]


def _same_batch(res, h, ores, oh, tag):
    for f in RESULT_FIELDS:
        if f == "tie_flags":
            continue
        assert np.array_equal(res[f], ores[f]), (tag, f, res[f][:4], ores[f][:4])
    assert np.array_equal(h, oh), tag


@pytest.mark.parametrize("ndev", [2, 3])
def test_replicas_split_over_shards(engine_mod, oracle_mod, ndev):
    scn = scenarios.token_ring(n_nodes=12, n_replicas=70, launch_duration=30_000_000, drop_log2=3, link_depth=2)
    with engine_mod.Engine(devices=[0] * ndev) as e:
        assert e.info() == (ndev, ndev, 0, 2)  # duplicate device: the copy transport
        e.load(scn)
        st = e.run()
        res, h = e.results(), e.hashes()
    ores, oh = oracle_mod.run_batch(scn, threads=8)
    _same_batch(res, h, ores, oh, f"ndev={ndev}")
    assert st.events == int(ores["events"].sum())
    assert st.replicas_done == scn.n_replicas


def test_lpb_split_over_shards(engine_mod, oracle_mod):
    # batched logical processes, a power-of-two block of replicas per shard
    scn = scenarios.hotspot(n_senders=16, n_replicas=64, msg_num=30)
    with engine_mod.Engine(devices=[0, 0]) as e:
        e.load(scn, geometry="lpb")
        st = e.run()
        res, h = e.results(), e.hashes()
    ores, oh = oracle_mod.run_batch(scn, threads=8)
    _same_batch(res, h, ores, oh, "lpb x2")
    assert st.events == int(ores["events"].sum())


@pytest.mark.parametrize("ndev,xcap", [(1, None), (2, None), (4, None), (4, 8)])
def test_lp_run_over_shards(engine_mod, oracle_mod, monkeypatch, ndev, xcap):
    """tw_lp_run: the library-driven device window loop over ndev shards (a
    record block of only 8 records makes most foreign records wait in the
    carry buffer, and the block size adapt)."""
    if xcap:
        monkeypatch.setenv("TW_LP_XCAP", str(xcap))
    scn = scenarios.gossip(6000, drop_log2=4, seed=21)
    L = int(scn.meta["lookahead_us"])
    s = engine_mod.lp_scenario(scn)
    with engine_mod.LPEngine(s, 0, scn.n_nodes, L, devices=[0] * ndev) as e:
        e.reset()
        lp = e.run_lp()
        agg, hashes = e.lp_results()
    o = oracle_mod.run(scn, trace_cap=0)
    for f in ("final_t", "events", "delivered", "dropped", "undeliverable", "status", "main_exc", "threads"):
        assert int(agg[f]) == int(o.result[f]), (ndev, xcap, f, int(agg[f]), o.result[f])
    assert np.array_equal(hashes, o.hashes)
    assert lp.done == 1 and lp.err == 0 and lp.windows > 1


def test_one_rank_rccl_replicas(engine_mod, oracle_mod):
    """A one-rank RCCL job: tw_run's statistics come back through the
    library's all-reduce."""
    jid = engine_mod.comm_id()
    scn = scenarios.token_ring(n_nodes=10, n_replicas=48, launch_duration=25_000_000, drop_log2=4)
    with engine_mod.Engine(0, comm=(1, 0, jid)) as e:
        assert e.info() == (1, 1, 0, 1)
        e.load(scn)
        st = e.run()
        res, h = e.results(), e.hashes()
        e.reset()
        st2 = e.run()
    ores, oh = oracle_mod.run_batch(scn, threads=8)
    _same_batch(res, h, ores, oh, "rccl x1")
    assert st.events == st2.events == int(ores["events"].sum())
    assert st.delivered == int(ores["delivered"].sum()) and st.dropped == int(ores["dropped"].sum())
    assert st.max_final_t == int(ores["final_t"].max())


def test_one_rank_rccl_lpb(engine_mod, oracle_mod):
    """bench.py's C3 at 8 GPUs: each rank runs its replica block as batched
    logical processes (tw_lpb_load on a tw_create_rank context); tw_run's
    statistics come back through the library's all-reduce."""
    jid = engine_mod.comm_id()
    scn = scenarios.token_ring(n_nodes=16, n_replicas=32, launch_duration=40_000_000, drop_log2=4)
    with engine_mod.Engine(0, comm=(1, 0, jid)) as e:
        e.load(scn, geometry="lpb")
        assert e.geometry() == "lpb"
        st = e.run()
        res, h = e.results(), e.hashes()
        e.reset()
        st2 = e.run()
    ores, oh = oracle_mod.run_batch(scn, threads=8)
    _same_batch(res, h, ores, oh, "rccl x1 lpb")
    assert st.events == st2.events == int(ores["events"].sum())
    assert st.delivered == int(ores["delivered"].sum()) and st.dropped == int(ores["dropped"].sum())
    assert st.max_final_t == int(ores["final_t"].max())


def test_one_rank_rccl_lp_loop(engine_mod, oracle_mod):
    """tw_lp_run over a one-rank RCCL communicator: the record blocks go
    through ncclSend/ncclRecv to itself, the window words through
    ncclAllReduce(min), the results and node hashes through the library's
    reductions -- and the scenario still equals the oracle, run twice."""
    jid = engine_mod.comm_id()
    scn = scenarios.gossip(5000, drop_log2=3, seed=9)
    L = int(scn.meta["lookahead_us"])
    s = engine_mod.lp_scenario(scn)
    o = oracle_mod.run(scn, trace_cap=0)
    with engine_mod.LPEngine(s, 0, scn.n_nodes, L, comm=(1, 0, jid)) as e:
        for _ in range(2):
            e.reset()
            lp = e.run_lp()
            agg, hashes = e.lp_results()
            for f in ("final_t", "events", "delivered", "dropped", "undeliverable", "status", "threads"):
                assert int(agg[f]) == int(o.result[f]), (f, int(agg[f]), o.result[f])
            assert np.array_equal(hashes, o.hashes)
            assert lp.done == 1 and lp.err == 0


@pytest.mark.parametrize("mode", ["copy", "rccl"])
def test_lp_run_local_failure_agreed(engine_mod, oracle_mod, monkeypatch, mode):
    """A failure local to one shard (injected: TW_TEST_FAIL_TICK=shard:tick
    fails that shard's launches at that tick, as a HIP error would) does not
    strand the others in the exchange: every shard keeps exchanging and
    reducing until the batch's agreement, and tw_lp_run returns the agreed
    code (TW_ERR_STATE) on all of them.  The next call sets the loop up again
    and runs the scenario to the oracle's result."""
    scn = scenarios.gossip(3000, drop_log2=4, seed=5)
    L = int(scn.meta["lookahead_us"])
    s = engine_mod.lp_scenario(scn)
    kw = dict(devices=[0, 0]) if mode == "copy" else dict(comm=(1, 0, engine_mod.comm_id()))
    with engine_mod.LPEngine(s, 0, scn.n_nodes, L, **kw) as e:
        e.reset()
        monkeypatch.setenv("TW_TEST_FAIL_TICK", "1:5" if mode == "copy" else "0:5")
        with pytest.raises(engine_mod.EngineError, match=r"tw_lp_run failed: -5 "):
            e.run_lp()
        monkeypatch.delenv("TW_TEST_FAIL_TICK")
        e.reset()
        lp = e.run_lp()
        agg, hashes = e.lp_results()
    o = oracle_mod.run(scn, trace_cap=0)
    for f in ("final_t", "events", "delivered", "dropped", "undeliverable", "status", "threads"):
        assert int(agg[f]) == int(o.result[f]), (mode, f, int(agg[f]), o.result[f])
    assert np.array_equal(hashes, o.hashes)
    assert lp.done == 1 and lp.err == 0


@pytest.mark.parametrize("k", [1, 2, 3, 4])
def test_rccl_failure_marks_the_context_unusable(engine_mod, oracle_mod, monkeypatch, k):
    """A failed RCCL call returns TW_ERR_COMM and marks the context: every
    later call that communicates returns TW_ERR_COMM at once instead of
    entering a collective its peers may no longer be in (include/timewarp.h,
    tw_lp_run).  Injected with TW_TEST_FAIL_NCCL=k, read when the context is
    made: its k-th checked RCCL call fails without being made -- tw_run's
    statistics reduction is ncclGroupStart (1), two ncclAllReduce calls (2, 3)
    and ncclGroupEnd (4), so k = 2, 3 fail inside the group, which the library
    must close before it returns, and k = 4 fails at the close itself.  The
    broken context is aborted (ncclCommAbort) at tw_destroy, and a fresh
    context made afterwards on the same thread -- its own group not folded
    into a half-open one -- works again."""
    scn = scenarios.token_ring(n_nodes=10, n_replicas=48, launch_duration=25_000_000, drop_log2=4)
    monkeypatch.setenv("TW_TEST_FAIL_NCCL", str(k))
    with engine_mod.Engine(0, comm=(1, 0, engine_mod.comm_id())) as e:
        monkeypatch.delenv("TW_TEST_FAIL_NCCL")  # (read once, at tw_create_rank)
        e.load(scn)
        with pytest.raises(engine_mod.EngineError, match=r"tw_run failed: -8 "):
            e.run()
        e.reset()
        with pytest.raises(engine_mod.EngineError, match=r"tw_run failed: -8 "):
            e.run()
    with engine_mod.Engine(0, comm=(1, 0, engine_mod.comm_id())) as e:
        e.load(scn)
        st = e.run()
        res, h = e.results(), e.hashes()
    ores, oh = oracle_mod.run_batch(scn, threads=8)
    _same_batch(res, h, ores, oh, "rccl x1 after a failed context")
    assert st.events == int(ores["events"].sum())


def test_multi_shard_refuses_caller_loop(engine_mod):
    """The caller-driven window primitives speak for one device only."""
    scn = scenarios.gossip(256, seed=1)
    s = engine_mod.lp_scenario(scn)
    with engine_mod.LPEngine(s, 0, scn.n_nodes, int(scn.meta["lookahead_us"]), devices=[0, 0]) as e:
        with pytest.raises(engine_mod.EngineError, match=r"failed: -5 "):
            e.loop_begin()
