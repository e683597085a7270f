"""Split a token-ring run into start-up / token phase / teardown and time each (GPU)."""
import json, os, sys, time
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "time-warp_amd"))
from timewarp import scenarios
from timewarp.engine import Engine

R = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
N = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
L = 120_000_000
scn = scenarios.token_ring(n_nodes=N, n_replicas=R, launch_duration=L, drop_log2=10)
e = Engine(0).load(scn)
out = {}
for rep in range(2):
    e.reset()
    prev = 0
    for name, t_end in [("startup<1s", 999_999), ("token<L", L - 1), ("teardown", (1 << 63) - 1)]:
        st = e.run(t_end=t_end)
        ms = float(e.launch_ms().sum())
        out[name] = dict(events=st.events, kernel_ms=ms, launches=st.launches, ev_per_s=st.events / (ms / 1e3) if ms else 0)
    print(json.dumps(out), flush=True)
