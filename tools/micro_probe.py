"""Micro-scenarios that isolate the per-event cost of the engine's machinery (GPU).

  timers  : K threads per replica, thread i loops `wait (for (i+1) µs)` -> one
            pop and two interpreted instructions per event, near queue only
  forkers : K threads loop `fork_ child; ` with `child = end` -> two pops per
            fork (child start, parent resume at +1 µs), slot alloc/free
  sleepers: like timers with a 20 s wait (far runs + HBM records)

Prints events/s per scenario. usage: python tools/micro_probe.py [replicas] [K]
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "time-warp_amd"))
import numpy as np  # noqa: E402
from timewarp.program import Program  # noqa: E402
from timewarp.scenario import Scenario, Topology  # noqa: E402
from timewarp.engine import Engine  # noqa: E402
from timewarp.timeunits import for_  # noqa: E402


def alu_scenario(R, n_iter):
    """main runs `n_iter` times {addi r0 1; jlt r0 r2 loop} without yielding:
    a pure interpreter loop (no events besides the final ones)."""
    p = Program()
    c = p.function("main")
    c.seti(0, 0).setk(2, n_iter) if hasattr(c, "setk") else c.seti(2, n_iter)
    loop = c.here()
    c.addi(0, 1).jlt(0, 2, loop)
    c.wait(for_(1))
    c.end()
    img = p.finalize()
    topo = Topology.from_out_lists(1, [[]])
    return Scenario(name="micro_alu", image=img, topo=topo, n_replicas=R, main_pc=img.pc_of("main"),
                    main_node=0, max_slots=8, queue_capacity=64, run_capacity=64, near_horizon_us=10_000_000)


def scenario(kind, R, K, T):
    p = Program()
    c = p.function("main")
    c.seti(0, 0).seti(2, K)
    loop = c.here()
    c.fork_("worker")
    c.addi(0, 1).jlt(0, 2, loop)
    c.end()
    c = p.function("worker")          # r0 = index
    c.addi(0, 1)
    top = c.here()
    if kind == "timers":
        c.wait_reg(0)
    elif kind == "sleepers":
        c.wait(for_(20_000_000))
    else:
        c.fork_("child")
    c.now(1).seti(2, T).jlt(1, 2, top)
    c.end()
    c = p.function("child")
    c.end()
    img = p.finalize()
    topo = Topology.from_out_lists(1, [[]])
    return Scenario(name=f"micro_{kind}", image=img, topo=topo, n_replicas=R, main_pc=img.pc_of("main"),
                    main_node=0, max_slots=2 * K + 8, queue_capacity=4 * K + 64, run_capacity=4 * K + 64,
                    near_horizon_us=10_000_000)


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    K = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    out = {}
    for kind, T in (("timers", 20_000), ("forkers", 10_000), ("sleepers", 2_000_000_000)):
        scn = scenario(kind, R, K, T)
        e = Engine(0).load(scn)
        best = None
        for _ in range(2):
            e.reset()
            st = e.run()
            ms = float(e.launch_ms().sum())
            best = ms if best is None else min(best, ms)
        out[kind] = dict(events=st.events, kernel_ms=round(best, 3), gev_per_s=round(st.events / best / 1e6, 3))
    n_iter = 200_000
    scn = alu_scenario(R, n_iter)
    e = Engine(0).load(scn)
    e.reset()
    e.run()
    e.reset()
    e.run()
    ms = float(e.launch_ms().sum())
    out["alu"] = dict(insns_per_lane=2 * n_iter, kernel_ms=round(ms, 3),
                      ns_per_insn=round(ms * 1e6 / (2 * n_iter), 2))
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
