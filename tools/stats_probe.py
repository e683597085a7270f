"""Per-phase event-path counters from the diagnostic build (lib/libtimewarp_stats.so, -DTW_STATS=1).

Runs the config-3 token ring in three phases (start-up t < 1 s, token phase t <
launchDuration, teardown) and prints, per committed pop, how often each path of
the event loop ran: record source (prefetched copy / HBM), record
writes (full / dead header), s_memtime cycle splits (pop phase, interpreter
loop, step + hash flush; cycles are per wave, summed over lanes), prefetches issued, hash atomics,
queue pushes by tier, interpreted instructions.  Also times each phase.

usage: TW_LIB=.../libtimewarp_stats.so python tools/stats_probe.py [replicas] [nodes]
"""
import ctypes as C
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ.setdefault("TW_LIB", os.path.join(ROOT, "time-warp_amd", "lib", "libtimewarp_stats.so"))
sys.path.insert(0, os.path.join(ROOT, "time-warp_amd"))
from timewarp import scenarios  # noqa: E402
from timewarp.engine import Engine  # noqa: E402

NAMES = ["pop", "superseded", "peek_pf", "peek_hbm", "put_hbm", "put_dead", "pf_issue", "hash_imm", "hash_flush",
         "near_push", "run_push", "far_push", "insn", "cyc_pop", "cyc_interp", "cyc_step_and_flush",
         "cyc_select", "cyc_fetch", "cyc_qpop", "cyc_commit", "cyc_prefetch", "cyc_terminal", "cyc_store", "cyc_hash",
         "cyc_spawn", "cyc_enqueue", "spawn", "alloc_ld", "iter", "cyc_send", "cyc_deliver", "cyc_due", "cyc_pro",
         "cyc_epi", "cyc_ip", "pass"]


def read(eng, heavy=False):
    """the counters of every lane (heavy=True: of heavy-inbox LP lanes alone)"""
    buf = (C.c_ulonglong * (2 * len(NAMES) + 8))()
    fn = eng.lib.tw_prof_read
    fn.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
    n = fn(eng.ctx, buf, 2 * len(NAMES) + 8, 1)
    if n < 0:
        raise RuntimeError(f"tw_prof_read: {n}")
    o = len(NAMES) if heavy else 0
    d = {k: buf[o + i] for i, k in enumerate(NAMES)}
    if n >= 2 * len(NAMES) + 6:  # tw_lp_batch's phase cycles (staging, dry run, scan, -, effects, tail)
        d["bat_phase_cyc"] = [buf[2 * len(NAMES) + j] for j in range(6)]
    return d


def main():
    if len(sys.argv) > 1 and sys.argv[1] == "gossip":  # config 4 on the device window loop, one context
        import numpy as np

        from timewarp.engine import LPEngine, lp_scenario

        N = int(sys.argv[2]) if len(sys.argv) > 2 else 1 << 20
        scn = scenarios.gossip(N, seed=0)
        eng = LPEngine(lp_scenario(scn), 0, N, int(scn.meta["lookahead_us"]), 0)
        read(eng)
        eng.reset()
        eng.exchange_setup(1, 0, np.array([0, N]))
        eng.loop_begin()
        st = eng.run_windows()
        d = read(eng)
        pops = max(d["pop"], 1)
        print(json.dumps({"phase": "gossip", "windows": st.windows, "ticks": st.ticks,
                          "lane_efficiency": d["pop"] / max(d["iter"], 1),
                          "per_pop": {k: round(v / pops, 4) for k, v in d.items() if k not in ("pop", "bat_phase_cyc")}, "counters": d}))
        return
    if len(sys.argv) > 1 and sys.argv[1] in ("lpb_hotspot", "lpb_token"):  # C5 / C3 as logical processes
        R = int(sys.argv[2]) if len(sys.argv) > 2 else (4096 if sys.argv[1] == "lpb_hotspot" else 8192)
        if sys.argv[1] == "lpb_token":
            scn = scenarios.token_ring(n_nodes=4096, n_replicas=R, launch_duration=120_000_000, drop_log2=10)
        else:
            S = int(sys.argv[3]) if len(sys.argv) > 3 else 256
            scn = scenarios.hotspot(n_senders=S, n_replicas=R, msg_num=1000)
        eng = Engine(0).load(scn, geometry="lpb")
        read(eng)
        eng.reset()
        st = eng.run()
        if sys.argv[1] == "lpb_hotspot":  # the receivers alone first (read() clears every counter)
            d = read(eng, heavy=True)
            pops = max(d["pop"], 1)
            print(json.dumps({"phase": "lpb_hotspot_receivers", "lane_efficiency": d["pop"] / max(d["iter"], 1),
                              "per_pop": {k: round(v / pops, 4) for k, v in d.items() if k not in ("pop", "bat_phase_cyc")},
                              "counters": d}))
            eng.reset()
            st = eng.run()
        d = read(eng)
        pops = max(d["pop"], 1)
        w, t = eng.lpb_windows()
        print(json.dumps({"phase": sys.argv[1], "events": st.events, "loop_ms": st.kernel_ms, "windows": w,
                          "ticks": t, "lane_efficiency": d["pop"] / max(d["iter"], 1),
                          "per_pop": {k: round(v / pops, 4) for k, v in d.items() if k not in ("pop", "bat_phase_cyc")}, "counters": d}))
        return
    if len(sys.argv) > 1 and sys.argv[1] == "hotspot":  # config 5: one phase per 0.25 s of virtual time
        R = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
        S = int(sys.argv[3]) if len(sys.argv) > 3 else 256
        scn = scenarios.hotspot(n_senders=S, n_replicas=R, msg_num=1000)
        phases = [("t<0.25s", 249_999), ("t<0.5s", 499_999), ("t<1s", 999_999), ("rest", (1 << 63) - 1)]
    else:
        R = int(sys.argv[1]) if len(sys.argv) > 1 else 65536
        N = int(sys.argv[2]) if len(sys.argv) > 2 else 4096
        Ld = 120_000_000
        scn = scenarios.token_ring(n_nodes=N, n_replicas=R, launch_duration=Ld, drop_log2=10)
        phases = [("startup<1s", 999_999), ("token<L", Ld - 1), ("teardown", (1 << 63) - 1)]
    eng = Engine(0).load(scn)
    if os.environ.get("TW_PROBE_TIE"):  # e.g. forkfirst (bench.py's C3 order)
        eng.set_tie_mode(os.environ["TW_PROBE_TIE"])
    if not hasattr(eng.lib, "tw_prof_read"):
        raise SystemExit("TW_LIB is not the diagnostic build (tw_prof_read missing)")
    read(eng)
    eng.reset()
    for name, t_end in phases:
        st = eng.run(t_end=t_end)
        d = read(eng)
        ms = float(eng.launch_ms().sum())
        pops = max(d["pop"], 1)
        rec = {"phase": name, "events": st.events, "kernel_ms": round(ms, 3),
               "ev_per_s": st.events / max(ms, 1e-9) * 1e3,
               "per_pop": {k: round(v / pops, 4) for k, v in d.items() if k not in ("pop", "bat_phase_cyc")}, "counters": d}
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
