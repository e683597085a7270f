"""HIP engine vs oracle on the reference's semantic pins (doc KATs,
ExceptionSpec cases, timeout/kill properties), C1 record-replay, and on
adversarial random fork/throwTo/catch/timeout programs — every output
bit-exact against the oracle's canonical mode, through the C ABI."""
import numpy as np
import pytest

import progs
from test_golden_c1 import GOLD, c1_table_scenario
from timewarp import isa
from timewarp.abi import RESULT_DTYPE, RESULT_FIELDS

pytestmark = pytest.mark.gpu

FIELDS = list(RESULT_FIELDS)


def _gpu(engine_mod, scn, t_end=None, max_events=None):
    kw = {}
    if t_end is not None:
        kw["t_end"] = t_end
    if max_events is not None:
        kw["max_events"] = max_events
    st, res, h = engine_mod.run_scenario(scn, **kw)
    return res, h


def _same(scn, res, h, ores, oh):
    for f in FIELDS:
        assert np.array_equal(res[f], ores[f]), (scn.name, f, res[f][:4], ores[f][:4])
    assert np.array_equal(h, oh), scn.name


@pytest.mark.parametrize("case", progs.KATS + progs.EXCEPTION_SPEC, ids=lambda f: getattr(f, "__name__", "exc"))
def test_spec_programs(engine_mod, oracle_mod, case):
    scn, _ = case()
    res, h = _gpu(engine_mod, scn)
    ores, oh = oracle_mod.run_batch(scn)
    _same(scn, res, h, ores, oh)


@pytest.mark.parametrize("tout,wt", [(0, 0), (1, 0), (2, 1), (5, 10), (10, 5), (7, 6), (1000, 999), (3, 3)])
def test_timeout(engine_mod, oracle_mod, tout, wt):
    scn = progs.timeout_prog(tout, wt)
    res, h = _gpu(engine_mod, scn)
    ores, oh = oracle_mod.run_batch(scn)
    _same(scn, res, h, ores, oh)


@pytest.mark.parametrize("m,f1,f2", [(0, 0, 0), (5, 3, 9), (9, 3, 5), (1, 2, 3), (100, 1, 1)])
def test_kill_thread(engine_mod, oracle_mod, m, f1, f2):
    scn = progs.kill_thread_prog(m, f1, f2)
    res, h = _gpu(engine_mod, scn)
    ores, oh = oracle_mod.run_batch(scn)
    _same(scn, res, h, ores, oh)


def test_work(engine_mod, oracle_mod):
    scn = progs.work_prog(life=10_000, period=700)
    res, h = _gpu(engine_mod, scn)
    ores, oh = oracle_mod.run_batch(scn)
    _same(scn, res, h, ores, oh)


@pytest.mark.parametrize("seed", range(48))
def test_random_programs(engine_mod, oracle_mod, seed):
    """Tie-heavy programs: GPU must follow the canonical (t, seq) order exactly,
    including error statuses (slot / timeout-epoch exhaustion) and a t_end cut."""
    scn = progs.random_program(seed)
    res, h = _gpu(engine_mod, scn, t_end=3000)
    o = oracle_mod.run(scn, t_end=3000)
    for f in FIELDS:
        assert res[f][0] == o.result[f], (seed, f, res[f][0], o.result[f])
    assert np.array_equal(h[0], o.hashes), seed


def test_c1_record_replay_on_gpu(engine_mod):
    scn = c1_table_scenario()
    res, h = _gpu(engine_mod, scn)
    for f in FIELDS:
        assert res[f][0] == GOLD["result"][f], f
    assert [f"{int(x):016x}" for x in h[0]] == GOLD["hashes"]


def test_run_in_pieces_equals_one_run(engine_mod, oracle_mod):
    """tw_run may be called repeatedly (t_end, then max_events, then to quiescence)."""
    from timewarp import scenarios
    from timewarp.engine import Engine

    scn = scenarios.token_ring(n_nodes=10, n_replicas=70, launch_duration=40_000_000, drop_log2=4, link_depth=4)
    with Engine() as e:
        e.load(scn)
        e.run(t_end=1_000_500)
        e.run(max_events=300)
        e.run(t_end=30_000_000)
        e.run()
        res, h = e.results(), e.hashes()
        e.reset()
        e.run()
        res2, h2 = e.results(), e.hashes()
    ores, oh = oracle_mod.run_batch(scn, threads=8)
    _same(scn, res, h, ores, oh)
    _same(scn, res2, h2, ores, oh)


def _cap_prog(kind: str, k: int):
    """A step that runs into the 2^22-instruction cap (TW_REP_ERR_INSN) or just
    fits under it, with the boundary on an instruction the run geometries fold
    into the pass before it (Lane::FOLD): the loop's jump after its
    `addi` (U_NJ) and its END after the loop (U_NE); or a `catch` followed by a
    wait (U_NW).  The folded step must count exactly as the oracle does."""
    from timewarp.program import Program
    from timewarp.timeunits import for_
    p = Program()
    c = p.function("main")
    c.seti(0, 0).seti(1, k)
    top = c.here()
    c.addi(0, 1).jlt(0, 1, top)
    if kind == "wait":
        c.catch_(1 << 4, "h")
        c.wait(for_(5))
        c.uncatch()
    c.end()
    c = p.function("h")
    c.end()
    return progs.single(p, name=f"cap_{kind}_{k}")


@pytest.mark.one_geometry
@pytest.mark.parametrize("geometry", ["dense", "compact"])
@pytest.mark.parametrize("kind,k", [("jump", 2097150), ("jump", 2097151), ("wait", 2097150), ("wait", 2097151)])
def test_step_cap_on_folded_instructions(engine_mod, oracle_mod, geometry, kind, k):
    scn = _cap_prog(kind, k)
    st, res, h = engine_mod.run_scenario(scn, geometry=geometry)
    o = oracle_mod.run(scn)
    for f in FIELDS:
        assert res[f][0] == o.result[f], (kind, k, f, res[f][0], o.result[f])
    assert np.array_equal(h[0], o.hashes)
    # 2 + 2k + 1 (END) or 2 + 2k + 2 (catch, wait) against the cap of 2^22
    n = 2 + 2 * k + (1 if kind == "jump" else 2)
    assert (int(o.result["status"]) == isa.REP_ERR_INSN) == (n > 1 << 22), (kind, k, o.result["status"])
