"""tw_lp_batch's phase cycles on C5 (diagnostic build, lib/libtimewarp_stats.so):
lane set-up + record loads, the dry run, the prefix scan, the slot replay, the
effects pass, the totals -- s_memtime cycles summed over the heavy lanes a
workgroup served, per window.

usage: TW_LIB=.../libtimewarp_stats.so python tools/batch_probe.py [senders] [replicas] [msgs]"""
import ctypes as C
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("TW_LIB", os.path.join(ROOT, "time-warp_amd", "lib", "libtimewarp_stats.so"))
sys.path.insert(0, os.path.join(ROOT, "time-warp_amd"))
from timewarp import scenarios  # noqa: E402
from timewarp.engine import Engine, draw_link_table  # noqa: E402

P_COUNT = 36
S, R, M = (int(x) for x in (sys.argv[1:4] + ["256", "4096", "1000"][len(sys.argv) - 1:]))
scn = scenarios.hotspot(n_senders=S, n_replicas=R, msg_num=M, drawer=draw_link_table)
with Engine(0) as e:
    e.load(scn, geometry="lpb")
    n = 2 * P_COUNT + 8
    buf = (C.c_ulonglong * n)()
    fn = e.lib.tw_prof_read
    fn.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    e.reset()
    fn(e.ctx, buf, n, 1)
    st = e.run()
    fn(e.ctx, buf, n, 1)
    w, t = e.lpb_windows()
    names = ["setup+loads", "dry_run", "scan", "replay", "effects", "totals"]
    cyc = {k: buf[2 * P_COUNT + i] for i, k in enumerate(names)}
    print({"events": st.events, "kernel_ms": st.kernel_ms, "windows": w, "batch": e.lpb_batch(),
           "cycles_per_lane_window": {k: round(v / max(1, w) / R, 1) for k, v in cyc.items()}})
