"""A/B of the scenario compiler (tw_set_jit) against the interpreter on one
workload: both engines run the same scenario, every replica's results and node
hashes must be identical; prints the step time of each.

usage: python tools/jit_probe.py [token_ring|ping_pong|hotspot] [replicas] [geometry]
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "time-warp_amd"))
from timewarp import scenarios  # noqa: E402
from timewarp.engine import Engine, draw_link_table  # noqa: E402
from timewarp.timeunits import sec  # noqa: E402


def build(cfg, R):
    if cfg == "token_ring":
        return scenarios.token_ring(4096, R, launch_duration=sec(120), drop_log2=10, drawer=draw_link_table)
    if cfg == "ping_pong":
        return scenarios.ping_pong(R, round_trips=1000, drawer=draw_link_table)
    return scenarios.hotspot(n_senders=256, n_replicas=R, msg_num=1000, drawer=draw_link_table)


def main():
    cfg = sys.argv[1] if len(sys.argv) > 1 else "token_ring"
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 65536
    geo = sys.argv[3] if len(sys.argv) > 3 else None
    steps = int(os.environ.get("JIT_PROBE_STEPS", "3"))
    scn = build(cfg, R)
    out = {"config": cfg, "replicas": R}
    res = {}
    for jit in (0, 1):
        eng = Engine(0)
        t0 = time.perf_counter()
        if jit:
            eng.set_jit(True)
        eng.load(scn, geometry=geo)
        load_s = time.perf_counter() - t0
        eng.reset()
        eng.run()  # warm-up
        ms = []
        for _ in range(steps):
            eng.reset()
            st = eng.run()
            ms.append(float(eng.launch_ms().sum()))
        r = eng.results()
        h = eng.hashes()
        res[jit] = (r, h)
        on, cms = eng.jit_status()
        out[f"jit{jit}"] = {"geometry": eng.geometry(), "jit_on": on, "compile_ms": cms, "load_s": round(load_s, 2),
                            "kernel_ms": [round(x, 2) for x in ms], "events": int(st.events),
                            "gev_s": round(st.events / (min(ms) / 1e3) / 1e9, 3)}
        print(json.dumps(out[f"jit{jit}"]), flush=True)
        eng.close()
    (r0, h0), (r1, h1) = res[0], res[1]
    same = all(np.array_equal(r0[f], r1[f]) for f in r0.dtype.names) and np.array_equal(h0, h1)
    out["identical"] = bool(same)
    out["speedup"] = round(min(out["jit0"]["kernel_ms"]) / min(out["jit1"]["kernel_ms"]), 3)
    print(json.dumps(out), flush=True)
    if not same:
        sys.exit(3)


if __name__ == "__main__":
    main()
