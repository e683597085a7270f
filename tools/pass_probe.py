"""Per-instruction cost of a hotspot receiver's chain: the C5 shape with k extra
trace instructions in the Ping handler (scenarios.hotspot(probe_traces=k)).
Prints the device window-loop time per run for each k; the slope over k and
the messages per receiver gives the cost of one interpreter pass on the chain.

usage: python tools/pass_probe.py [senders] [replicas] [msgs] [geometry] [trace|load]
(geometry: lpb -- the default -- or a replica geometry: dense, narrow, ...; in a
replica geometry a lane runs the whole replica, so the slope is per message of
the replica, senders' work included)
"""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "time-warp_amd"))
from timewarp import scenarios  # noqa: E402
from timewarp.engine import Engine  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 64
R = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
M = int(sys.argv[3]) if len(sys.argv) > 3 else 200
G = sys.argv[4] if len(sys.argv) > 4 else "lpb"
KIND = sys.argv[5] if len(sys.argv) > 5 else "trace"
KS = [int(x) for x in os.environ.get("PROBE_KS", "0,4,16").split(",")]
for k in KS:
    extra = {"probe_traces": k} if KIND == "trace" else {"probe_loads": k}
    scn = scenarios.hotspot(n_senders=S, n_replicas=R, msg_num=M, **extra)
    eng = Engine(0).load(scn, geometry=G)
    best = None
    for _ in range(int(os.environ.get("PROBE_REPS", "3"))):
        eng.reset()
        st = eng.run()
        best = st.kernel_ms if best is None else min(best, st.kernel_ms)
    w = eng.lpb_windows()[0] if G == "lpb" else 1
    # lpb: µs per message of the receiver's chain (per window); replica
    # geometries: µs per message of a replica (the whole run is one chain)
    per_msg = best * 1e3 / max(w, 1) / S if G == "lpb" else best * 1e3 / (S * M)
    print(json.dumps({"geometry": G, "extra": KIND, "extra_traces": k, "senders": S, "replicas": R, "msgs": M, "loop_ms": best,
                      "windows": w, "events": st.events, "us_per_msg": per_msg}), flush=True)
    eng.close()
