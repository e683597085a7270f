"""Generate tests/golden/*.json from the oracle (committed; rerun only on a
deliberate semantics change).

token_ring_c1.json — BASELINE.json config 1: examples/token-ring under TimedT
pure emulation, 16 nodes, launchDuration 20 s, Delays drawn from ONE live
`mkStdGen 0` generator in pop order (examples/token-ring/Main.hs:60,73-77),
canonical queue order.  Also records the per-(link, ordinal) draws so the GPU
can replay them as a link table (record-replay).
"""
import json
import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
sys.path[:0] = [os.path.join(ROOT, "time-warp_amd"), os.path.join(ROOT, "oracle")]

import oracle  # noqa: E402
from timewarp import scenarios  # noqa: E402

DEPTH = 4


def c1():
    scn = scenarios.token_ring(n_nodes=16, n_replicas=1, launch_duration=20_000_000)
    r = oracle.run(scn, 0, live_seed=0, record_depth=DEPTH)
    return {
        "config": "token-ring 16 nodes, launchDuration 20 s, mkStdGen 0 live Delays, canonical order",
        "result": r.result,
        "hashes": [f"{int(h):016x}" for h in r.hashes],
        "traces": [list(t) for t in r.traces],
        "record_depth": DEPTH,
        "recorded_table": r.recorded_table.tolist(),
    }


if __name__ == "__main__":
    with open(os.path.join(HERE, "token_ring_c1.json"), "w") as f:
        json.dump(c1(), f, indent=1)
    print("wrote token_ring_c1.json")
