"""throwTo run back to back (TimedT.hs:357-368, MonadTimed.hs:205-206) on
every replica geometry against the oracle: two victims, one victim twice (the
first exception wins), main itself then a victim, a dead thread then a victim,
and a jump into the middle of a run -- the shapes of token-ring's teardown
(`killThread r1 >> killThread r2`)."""
import numpy as np
import pytest

from timewarp.abi import RESULT_FIELDS
from timewarp.program import Program
from timewarp.scenario import Scenario, Topology
from timewarp.timeunits import for_


def _gpu_run(engine_mod, scn, geometry=None):
    with engine_mod.Engine(0) as e:
        e.load(scn, geometry=geometry)
        e.reset()
        e.run()
        return e.results(), e.hashes()


def _throw_prog(case):
    """main forks two victims that catch USER0/USER1 (tracing value and code)
    and sleep; then runs of THROW_TOs -- two victims, one victim twice (first
    exception wins), main itself then a victim, a dead thread then a victim,
    and (case "jump") a second lap that jumps into the middle of a run."""
    from timewarp.isa import EXC_USER0
    E0, E1 = EXC_USER0, EXC_USER0 + 1
    p = Program()
    c = p.function("main")
    c.catch_((1 << E0) | (1 << E1), "main_h")
    c.fork("victim", ref=1).fork("victim", ref=2).fork("quick", ref=3)
    c.wait(for_(10))
    c.seti(0, 5)
    lap = p.label("lap")
    p.bind(lap)
    c.throw_to(1, E0, 0).throw_to(2, E1, 0)        # two victims
    c.wait(for_(10))
    c.addi(0, 1).throw_to(1, E1, 0)
    second = p.label("second")
    p.bind(second)
    c.throw_to(1, E0, 0)                           # one victim twice
    c.wait(for_(10))
    if case == "self":
        c.my_thread_id(3).throw_to(3, E1, 0).throw_to(2, E0, 0)   # main itself, then a victim
    else:
        c.throw_to(3, E0, 0).throw_to(2, E0, 0)    # a dead thread, then a victim
    c.wait(for_(10))
    if case == "jump":
        c.addi(0, 10).jnei(0, 16, "lap_end").jmp(second)   # one more lap from the pair's second half
        p.bind(p.label("lap_end"))
    c.kill_thread(1).kill_thread(2)                # (the victims end: a pair too)
    c.end()
    h = p.function("main_h")
    h.trace(9, 0).trace(10, 3).kill_thread(1).kill_thread(2).end()
    v = p.function("victim")
    v.catch_((1 << E0) | (1 << E1), "victim_h")
    v.sleep_forever()
    vh = p.function("victim_h")
    vh.trace(7, 0).trace(8, 3).jmp("victim")
    q = p.function("quick")
    q.end()
    img = p.finalize()
    topo = Topology.from_out_lists(1, [[]])
    return Scenario(name="throw_pairs", image=img, topo=topo, n_replicas=2, main_pc=img.pc_of("main"), main_node=0,
                    max_slots=8, queue_capacity=64, run_capacity=16, max_timeouts=2, max_frames=4)



@pytest.mark.gpu
@pytest.mark.one_geometry
@pytest.mark.parametrize("geometry", [None, "dense", "sparse", "wave", "narrow", "compact", "half"])
@pytest.mark.parametrize("case", ["plain", "self", "jump"])
def test_gpu_throw_sequences(engine_mod, oracle_mod, case, geometry):
    """throwTo runs back to back (two victims, one victim twice -- the first
    exception wins --, main itself, a dead thread, a jump into the middle of a
    run), every geometry, against the oracle."""
    scn = _throw_prog(case)
    rf, hf = _gpu_run(engine_mod, scn, geometry)
    ro, ho = oracle_mod.run_batch(scn, threads=1)
    for f in RESULT_FIELDS:
        if f == "tie_flags":
            continue
        assert np.array_equal(rf[f], ro[f]), (f, rf[f], ro[f])
    assert np.array_equal(hf, ho)


