"""Full-batch oracle parity on the benched shapes.

bench.py checks a ~10-s sample of each batch against the oracle; this runs the
WHOLE batch once on the GPU exactly as bench.py does (same builders, device-
drawn link tables, geometry and tie order) and compares EVERY replica with
the oracle's canonical (t, seq) run (oracle/timedt_oracle.cpp, TimedT.hs:
234-304): every result field and every per-node trace hash.

  C3  token ring 4,096 nodes x 65,536 replicas, drop 2^-10, 120 s (dense,
      FORKFIRST -- the bench's order -- against the canonical oracle)
  C2  ping-pong 2 nodes x 1,048,576 replicas, 1,000 round trips (compact)
  C5  hotspot 256 senders -> 1 x 4,096 replicas, 1,000 messages (lpb, with
      the data-parallel due-run batch tw_lp_batch on)

usage: python tools/parity_all.py [c3|c2|c5 ...] [--threads N] [--chunk N]
Writes one JSON line per config (and progress lines to stderr every chunk, so
a long oracle run is never silent); exit 1 on any mismatch.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "time-warp_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))

import numpy as np  # noqa: E402


def build(cfg, drawer):
    from timewarp import scenarios

    if cfg == "c3":
        return scenarios.token_ring(n_nodes=4096, n_replicas=65536, launch_duration=120_000_000, drop_log2=10,
                                    drawer=drawer), None, "forkfirst"
    if cfg == "c2":
        return scenarios.ping_pong(n_replicas=1 << 20, round_trips=1000, drawer=drawer), None, "fifo"
    if cfg == "c5":
        return scenarios.hotspot(n_senders=256, n_replicas=4096, msg_num=1000, drawer=drawer), "lpb", "fifo"
    raise SystemExit(f"unknown config {cfg}")


def check(cfg, threads, chunk):
    import functools

    import oracle  # the parity checker
    from timewarp.abi import RESULT_FIELDS
    from timewarp.engine import Engine, draw_link_table

    t0 = time.perf_counter()
    scn, geo, tie = build(cfg, functools.partial(draw_link_table, device=0))
    with Engine(0) as e:
        e.load(scn, geometry=geo)
        if tie != "fifo":
            e.set_tie_mode(tie)
        e.reset()
        st = e.run()
        res, hashes = e.results(), e.hashes()
        geometry = e.geometry()
        bat = e.lpb_batch() if geometry == "lpb" else None
    gpu_s = time.perf_counter() - t0
    R = scn.n_replicas
    print(f"[parity_all] {cfg}: GPU {st.events} events over {R} replicas ({geometry}, {tie}) in {gpu_s:.1f} s",
          file=sys.stderr, flush=True)
    bad_fields = {f: 0 for f in RESULT_FIELDS if f != "tie_flags"}
    bad_hash_reps = 0
    first_bad = None
    oracle_events = 0
    t1 = time.perf_counter()
    for r0 in range(0, R, chunk):
        r1 = min(R, r0 + chunk)
        ores, oh = oracle.run_batch(scn, r0, r1, threads=threads)
        oracle_events += int(ores["events"].sum())
        for f in bad_fields:
            m = np.nonzero(res[f][r0:r1] != ores[f])[0]
            bad_fields[f] += int(m.size)
            if m.size and first_bad is None:
                first_bad = {"replica": r0 + int(m[0]), "field": f, "gpu": int(res[f][r0 + m[0]]),
                             "oracle": int(ores[f][m[0]])}
        hm = np.nonzero((hashes[r0:r1] != oh).any(axis=1))[0]
        bad_hash_reps += int(hm.size)
        if hm.size and first_bad is None:
            first_bad = {"replica": r0 + int(hm[0]), "field": "hashes",
                         "nodes": np.nonzero(hashes[r0 + hm[0]] != oh[hm[0]])[0][:8].tolist()}
        print(f"[parity_all] {cfg}: replicas [{r0}, {r1}) checked, {time.perf_counter() - t1:.1f} s, "
              f"mismatching so far: fields {sum(bad_fields.values())}, hash rows {bad_hash_reps}",
              file=sys.stderr, flush=True)
    ok = sum(bad_fields.values()) == 0 and bad_hash_reps == 0 and oracle_events == int(st.events)
    out = {"config": cfg, "replicas": R, "nodes": scn.n_nodes, "geometry": geometry, "tie_order": tie,
           "against": "oracle canonical (t, seq) order, every replica, every field, every node hash",
           "gpu_events": int(st.events), "oracle_events": oracle_events,
           "mismatching_replicas_by_field": bad_fields, "mismatching_hash_rows": bad_hash_reps,
           "first_mismatch": first_bad, "bit_exact": bool(ok), "oracle_threads": threads,
           "oracle_s": round(time.perf_counter() - t1, 1), "gpu_s": round(gpu_s, 1)}
    if bat is not None:
        out["lp_batch"] = {"batched_due_records": int(bat[0]), "due_records": int(bat[1])}
    print(json.dumps(out), flush=True)
    return ok


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("configs", nargs="*", default=["c3", "c2", "c5"])
    ap.add_argument("--threads", type=int, default=0, help="oracle threads (default: nproc)")
    ap.add_argument("--chunk", type=int, default=8192, help="replicas per oracle call (one progress line each)")
    a = ap.parse_args()
    threads = a.threads
    if threads <= 0:
        sys.path.insert(0, ROOT)
        from bench import host_cpu

        threads = host_cpu()[0]
    ok = True
    for cfg in a.configs:
        ok = check(cfg, threads, a.chunk if cfg != "c2" else max(a.chunk, 65536)) and ok
    sys.exit(0 if ok else 1)


if __name__ == "__main__":
    main()
