"""The scenario compiler (tw_set_jit, time-warp_amd/csrc/jit.cpp) against the
oracle (canonical mode) and against the interpreter: every output field and
every node hash bit-exact, through the C ABI.

Each compile takes seconds (hiprtc, in process), so this file picks programs
that together reach every instruction class: the BASELINE scenarios at their
shapes (token ring C3 4,096 nodes x 120 s with drops, ping-pong C2, hotspot
C5, gossip C4 and the batched logical processes), the reference's doc KATs and
ExceptionSpec cases, timeouts, killThread, and random fork/throwTo/catch
programs."""
import numpy as np
import pytest

import progs
from timewarp import scenarios
from timewarp.abi import RESULT_FIELDS
from timewarp.engine import Engine

pytestmark = [pytest.mark.gpu, pytest.mark.one_geometry]

FIELDS = list(RESULT_FIELDS)


def _run(scn, jit, geometry=None, t_end=None):
    with Engine(0) as e:
        if jit:
            e.set_jit(True)
        e.load(scn, geometry=geometry)
        on, _ = e.jit_status()
        assert on == bool(jit), "the compiled kernel did not load"
        st = e.run(t_end) if t_end is not None else e.run()
        return st, e.results(), e.hashes(), e.geometry()


def _same(name, a, b):
    (ra, ha), (rb, hb) = a, b
    bad = [f for f in FIELDS if not np.array_equal(ra[f], rb[f])]
    assert not bad, (name, bad, [(ra[f][:4], rb[f][:4]) for f in bad])
    assert np.array_equal(ha, hb), name


def _vs_oracle(scn, oracle_mod, geometry=None, t_end=None):
    st, res, h, geo = _run(scn, True, geometry, t_end)
    if geometry not in (None, "lpb"):
        assert geo == geometry
    if t_end is None:
        ores, oh = oracle_mod.run_batch(scn, threads=8)
    else:  # a t_end cut: replica by replica
        runs = [oracle_mod.run(scn, replica=r, t_end=t_end) for r in range(scn.n_replicas)]
        ores = np.zeros(scn.n_replicas, res.dtype)
        for r, o in enumerate(runs):
            for f in FIELDS:
                ores[f][r] = o.result[f]
        oh = np.stack([o.hashes for o in runs])
    _same(scn.name, (res, h), (ores, oh))
    return st, res, h


@pytest.mark.parametrize("geometry", ["dense", "narrow", "compact", "sparse", "half"])
def test_jit_token_ring_c3_shape(engine_mod, oracle_mod, geometry):
    """C3's node count, launchDuration and drop nastiness (4,096 nodes x 120 s,
    drop 2^-10), 16 replicas: compiled == oracle == interpreter."""
    scn = scenarios.token_ring(4096, 16, launch_duration=120_000_000, drop_log2=10)
    st, res, h = _vs_oracle(scn, oracle_mod, geometry)
    _, ri, hi, _ = _run(scn, False, geometry)
    _same("interp", (res, h), (ri, hi))
    assert st.events == int(res["events"].sum()) and (res["status"] == 1).all()


def test_jit_token_ring_drops_long(engine_mod, oracle_mod):
    scn = scenarios.token_ring(n_nodes=12, n_replicas=300, launch_duration=200_000_000, drop_log2=4, link_depth=8)
    _, res, _ = _vs_oracle(scn, oracle_mod, "dense")
    assert res["dropped"].sum() > 0


@pytest.mark.parametrize("geometry", ["compact", "dense"])
def test_jit_ping_pong(engine_mod, oracle_mod, geometry):
    _vs_oracle(scenarios.ping_pong(n_replicas=1000, round_trips=50), oracle_mod, geometry)


@pytest.mark.parametrize("geometry", ["sparse", "narrow"])
def test_jit_hotspot(engine_mod, oracle_mod, geometry):
    _vs_oracle(scenarios.hotspot(n_senders=8, n_replicas=130, msg_num=40), oracle_mod, geometry)


def test_jit_gatekeeper_raw_listener(engine_mod, oracle_mod):
    _vs_oracle(scenarios.gatekeeper(n_clients=6, n_replicas=200, msg_num=24, junk_every=3), oracle_mod, "dense")


def test_jit_socket_state(engine_mod, oracle_mod):
    _vs_oracle(scenarios.socket_state(n_replicas=64), oracle_mod, "dense")


def test_jit_spec_programs(engine_mod, oracle_mod):
    """Every doc KAT and ExceptionSpec program (one compile each)."""
    for case in progs.KATS + progs.EXCEPTION_SPEC:
        scn, _ = case()
        _vs_oracle(scn, oracle_mod, "dense")


@pytest.mark.parametrize("tout,wt", [(0, 0), (2, 1), (10, 5), (3, 3)])
def test_jit_timeout(engine_mod, oracle_mod, tout, wt):
    _vs_oracle(progs.timeout_prog(tout, wt), oracle_mod, "dense")


def test_jit_kill_thread(engine_mod, oracle_mod):
    _vs_oracle(progs.kill_thread_prog(5, 3, 9), oracle_mod, "narrow")


@pytest.mark.parametrize("seed", [0, 7, 19, 33])
def test_jit_random_programs(engine_mod, oracle_mod, seed):
    scn = progs.random_program(seed)
    _vs_oracle(scn, oracle_mod, "dense", t_end=3000)
