"""Per-phase kernel counters from the diagnostic build (lib/libtimewarp_prof.so, -DTW_PROF=1).

Runs the config-3 token ring in three phases, like tools/phase_probe.py: start-up (t < 1 s),
token phase (t < launchDuration) and teardown. After each phase it prints the counters the
kernel summed per wave: pops by queue source, record-cache hits and misses, write-backs,
hash flushes, interpreted instructions and waterfall passes, and s_memtime cycle splits
(select+pop / record wait / step). Per-op passes and cycles are printed too. Cycles are
per wave; divide by waves x pops-per-lane to get cycles per event.

usage: python tools/kernel_probe.py [replicas] [nodes]
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("TW_LIB", os.path.join(ROOT, "time-warp_amd", "lib", "libtimewarp_prof.so"))
sys.path.insert(0, os.path.join(ROOT, "time-warp_amd"))
from timewarp import isa, scenarios  # noqa: E402
from timewarp.engine import Engine  # noqa: E402

NAMES = ["loop_cyc", "sel_cyc", "wait_cyc", "step_cyc", "iters", "pops", "superseded", "src_near", "src_far",
         "src_run", "hit", "miss", "writeback", "hash_flush", "near_push", "run_push", "far_push", "insns",
         "passes", "active_lanes", "kernel_cyc", "prolog_cyc", "epilog_cyc", "hash_terms"]
OPS = {v: k[3:] for k, v in vars(isa).items() if k.startswith("OP_") and isinstance(v, int) and k != "OP_COUNT"}


def read(eng):
    buf = (C.c_ulonglong * 128)()
    fn = eng.lib.tw_prof_read
    fn.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    n = fn(eng.ctx, buf, 128, 1)
    if n < 0:
        raise RuntimeError(f"tw_prof_read: {n}")
    v = list(buf)
    out = {k: v[i] for i, k in enumerate(NAMES)}
    out["ops"] = {OPS.get(o, str(o)): {"passes": v[32 + o], "cyc": v[80 + o]} for o in range(43)
                  if v[32 + o] or v[80 + o]}
    return out


def derived(d, waves):
    it = max(d["iters"], 1)
    pops = max(d["pops"], 1)
    return {
        "cyc_per_iter": d["loop_cyc"] / it,
        "sel_per_iter": d["sel_cyc"] / it,
        "wait_per_iter": d["wait_cyc"] / it,
        "step_per_iter": d["step_cyc"] / it,
        "lanes_per_iter": d["active_lanes"] / it,
        "hit_rate": d["hit"] / max(d["hit"] + d["miss"], 1),
        "passes_per_iter": d["passes"] / it,
        "insns_per_pop": d["insns"] / pops,
        "src_mix": [d["src_near"] / pops, d["src_run"] / pops, d["src_far"] / pops],
        "kernel_cyc_per_wave": d["kernel_cyc"] / max(waves, 1),
    }


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    Ld = 120_000_000
    scn = scenarios.token_ring(n_nodes=N, n_replicas=R, launch_duration=Ld, drop_log2=10)
    eng = Engine(0).load(scn)
    if not hasattr(eng.lib, "tw_prof_read"):
        raise SystemExit("TW_LIB is not the diagnostic build (tw_prof_read missing)")
    waves = (R + 63) // 64
    read(eng)
    eng.reset()
    for name, t_end in [("startup<1s", 999_999), ("token<L", Ld - 1), ("teardown", (1 << 63) - 1)]:
        st = eng.run(t_end=t_end)
        d = read(eng)
        ms = float(eng.launch_ms().sum())
        rec = {"phase": name, "events": st.events, "kernel_ms": ms, "launches": st.launches,
               "derived": derived(d, waves * st.launches), "counters": d}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
