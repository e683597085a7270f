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

NAMES = ["sel_cyc", "wait_cyc", "pre_cyc", "step_cyc", "iters", "pops", "superseded", "src_near", "src_far",
         "src_run", "hit", "miss", "insns", "passes", "near_push", "run_push", "far_push", "hash", "store",
         "throwto", "alloc", "die", "loop_cyc", "tail_cyc", "store_cyc"]



LITE = ["sel_cyc", "pre_cyc", "step_cyc", "loop_cyc", "iters", "pops", "dispatch_cyc", "tail_cyc", "store_cyc", "spawn_cyc", "yenq_cyc", "throw_cyc", "die_cyc", "selmin_cyc", "load_cyc", "pop_cyc"]


def read(eng):
    buf = (C.c_ulonglong * 32)()
    fn = eng.lib.tw_prof_read
    fn.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    n = fn(eng.ctx, buf, 32, 1)
    if n < 0:
        raise RuntimeError(f"tw_prof_read: {n}")
    if os.environ.get("TW_PROBE_LITE"):
        return {k: buf[i] for i, k in enumerate(LITE)}
    return {k: buf[i] for i, k in enumerate(NAMES)}


def derived_lite(d):
    pops, it = max(d["pops"], 1), max(d["iters"], 1)
    return {"loop_per_pop": d["loop_cyc"] / pops, "sel_per_iter": d["sel_cyc"] / it,
            "pre_per_pop": d["pre_cyc"] / pops, "step_per_pop": d["step_cyc"] / pops,
            "iters_per_pop": it / pops, "dispatch_per_pop": d["dispatch_cyc"] / pops,
            "tail_per_pop": d["tail_cyc"] / pops, "store_per_pop": d["store_cyc"] / pops,
            **{k[:-4] + "_per_pop": d[k] / pops for k in ("spawn_cyc", "yenq_cyc", "throw_cyc", "die_cyc", "selmin_cyc",
                                                        "load_cyc", "pop_cyc")}}


def derived(d):
    """Counters are summed over lanes, cycles weighted by the lanes active in each
    iteration: x / pops = wave cycles (or counts) per committed event."""
    pops = max(d["pops"], 1)
    it = max(d["iters"], 1)
    return {
        "cyc_per_pop": d["loop_cyc"] / pops,
        "sel_per_iter": d["sel_cyc"] / it,
        "wait_per_iter": d["wait_cyc"] / it,
        "pre_per_pop": d["pre_cyc"] / pops,
        "step_per_pop": d["step_cyc"] / pops,
        "tail_per_pop": d["tail_cyc"] / pops,
        "store_per_pop": d["store_cyc"] / pops,
        "hit_rate": d["hit"] / max(d["hit"] + d["miss"], 1),
        "passes_per_pop": d["passes"] / pops,
        "insns_per_pop": d["insns"] / pops,
        "src_mix_near_run_far": [d["src_near"] / it, d["src_run"] / it, d["src_far"] / it],
        "per_pop": {k: d[k] / pops for k in ("hash", "store", "throwto", "alloc", "die", "near_push", "run_push",
                                             "far_push", "superseded", "miss")},
    }


def main():
    R = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
    N = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
    Ld = 120_000_000
    scn = scenarios.token_ring(n_nodes=N, n_replicas=R, launch_duration=Ld, drop_log2=10)
    eng = Engine(0).load(scn)
    if not hasattr(eng.lib, "tw_prof_read"):
        raise SystemExit("TW_LIB is not the diagnostic build (tw_prof_read missing)")
    read(eng)
    eng.reset()
    for name, t_end in [("startup<1s", 999_999), ("token<L", Ld - 1), ("teardown", (1 << 63) - 1)]:
        st = eng.run(t_end=t_end)
        d = read(eng)
        ms = float(eng.launch_ms().sum())
        rec = {"phase": name, "events": st.events, "kernel_ms": ms, "launches": st.launches,
               "ev_per_s": st.events / max(ms, 1e-9) * 1e3, "derived": derived_lite(d) if os.environ.get("TW_PROBE_LITE") else derived(d),
               "counters": d}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
