"""Debug: a hotspot batch at lp_max_slots=1 under the batched-LP kernels."""
import copy
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "time-warp_amd"))
import numpy as np  # noqa: E402
from timewarp import scenarios  # noqa: E402
from timewarp.engine import Engine, EngineError  # noqa: E402

slots = int(sys.argv[1]) if len(sys.argv) > 1 else 1
base = scenarios.hotspot(n_senders=64, n_replicas=16, msg_num=40)
scn = copy.copy(base)
scn.meta = dict(base.meta, lp_max_slots=slots)
with Engine(0) as e:
    e.load(scn, geometry="lpb")
    e.reset()
    try:
        st = e.run()
        print("run ok", st.events)
    except EngineError as x:
        print("run error", x)
    r = e.results()
    print("status", np.unique(r["status"], return_counts=True), "events", r["events"][:4], "delivered",
          r["delivered"][:4], "batch", e.lpb_batch())
