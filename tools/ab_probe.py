"""A/B of two engine settings on one workload: both run the same scenario,
every replica's results and node hashes must be identical (for a tie-order
A/B that holds when the workload is tie-insensitive); prints each setting's
kernel time per step.

usage: python tools/ab_probe.py CONFIG REPLICAS GEOMETRY SETTING_A SETTING_B
  CONFIG: token_ring | ping_pong | hotspot;  GEOMETRY: a geometry or "auto"
  SETTING: comma list of tie=fifo|lifo|forkfirst   e.g.  tie=fifo tie=lifo
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


def run(scn, geo, setting, steps):
    kv = dict(x.split("=") for x in setting.split(",") if x)
    eng = Engine(0)
    t0 = time.perf_counter()
    eng.load(scn, geometry=None if geo == "auto" else geo)
    load_s = time.perf_counter() - t0
    if "tie" in kv:
        eng.set_tie_mode(kv["tie"])
    eng.reset()
    eng.run()  # warm-up
    ms = []
    for _ in range(steps):
        eng.reset()
        st = eng.run()
        ms.append(float(eng.launch_ms().sum()))
    r, h = eng.results(), eng.hashes()
    out = {"setting": setting, "geometry": eng.geometry(), "load_s": round(load_s, 2),
           "kernel_ms": [round(x, 2) for x in ms], "events": int(st.events),
           "gev_s": round(st.events / (min(ms) / 1e3) / 1e9, 3), "errors": int(st.replicas_error)}
    eng.close()
    return out, r, h


def main():
    cfg, R, geo, a, b = sys.argv[1], int(sys.argv[2]), sys.argv[3], sys.argv[4], sys.argv[5]
    steps = int(os.environ.get("AB_STEPS", "3"))
    scn = build(cfg, R)
    oa, ra, ha = run(scn, geo, a, steps)
    print(json.dumps(oa), flush=True)
    ob, rb, hb = run(scn, geo, b, steps)
    print(json.dumps(ob), flush=True)
    fields = [f for f in ra.dtype.names if f != "tie_flags"]
    diff = {f: int((ra[f] != rb[f]).sum()) for f in fields if not np.array_equal(ra[f], rb[f])}
    hd = int((ha != hb).any(axis=1).sum())
    res = {"config": cfg, "replicas": R, "identical": not diff and hd == 0, "field_diffs": diff, "hash_diffs": hd,
           "speedup": round(min(oa["kernel_ms"]) / min(ob["kernel_ms"]), 3)}
    print(json.dumps(res), flush=True)
    if not res["identical"]:
        sys.exit(3)


if __name__ == "__main__":
    main()
