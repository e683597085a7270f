#!/usr/bin/env python3
"""Benchmark: committed events/s of the batched TimedT emulator (+ % HBM roofline).

Default workload = BASELINE.json config 3: token-ring, 4096 nodes, 65,536
replicas per GPU, network delay U[1 ms, 5 ms], drop 2^-10 per send
(examples/token-ring/Main.hs lowered).  One "step" = reset every
replica on the device-resident tables and run all of them to quiescence
(runTimedT, src/Control/TimeWarp/Timed/TimedT.hs:293-304).  An event = one
PQ.minView pop of the TimedT schedule (TimedT.hs:242); the GPU count equals the
oracle's (parity-checked on a sample each run).

Multi-GPU: one process per GPU (torchrun), replicas sharded in contiguous
blocks with no data-path collective (weak scaling: replicas per GPU fixed);
only the statistics are all-reduced over RCCL.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "time-warp_amd"))

import numpy as np  # noqa: E402

HBM_PEAK_GBS = 8000.0           # MI355X HBM3E peak (MI355X_MICROARCH.md)
BYTES_PER_EVENT = 64            # 16 B event read + 16 B event write + 32 B thread/node state r/w
BYTES_PER_SEND = 8              # link-table entry + ordinal


def build_scenario(args, rank: int):
    from timewarp import scenarios

    from timewarp.dist import weak_block

    base, R = weak_block(rank, args.replicas)
    if args.config == "token_ring":
        return scenarios.token_ring(n_nodes=args.nodes, n_replicas=R, launch_duration=args.duration_s * 1_000_000,
                                    drop_log2=args.drop_log2, seed_base=base), (
            f"token-ring (examples/token-ring) {args.nodes} nodes x {R} replicas/GPU, delay U[1,5] ms, "
            f"drop 2^-{args.drop_log2}, launchDuration {args.duration_s} s")
    if args.config == "ping_pong":
        return scenarios.ping_pong(n_replicas=R, round_trips=args.round_trips, seed_base=base), (
            f"ping-pong (examples/ping-pong) 2 nodes x {R} replicas/GPU, {args.round_trips} round trips, "
            "per-link delay U[1,5] ms")
    if args.config == "hotspot":
        return scenarios.hotspot(n_senders=args.nodes, n_replicas=R, msg_num=args.msg_num, seed_base=base), (
            f"hotspot (bench/Network) {args.nodes} senders -> 1 receiver x {R} replicas/GPU, "
            f"{args.msg_num} msgs @1000/s")
    if args.config == "gossip":
        return scenarios.gossip(n_nodes=args.nodes, seed=0), (
            f"gossip (config 4) one scenario of {args.nodes} nodes, fanout 4, delay U[1,5] ms, "
            f"node-partitioned over the GPUs, lookahead 1 ms windows")
    raise SystemExit(f"unknown config {args.config}")


def cpu_baseline(scn, gpu_res, gpu_hashes, seconds: float):
    """Oracle (C++ TimedT restatement, canonical mode) on host cores, bounded sample."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # the parity checker / CPU baseline — never the measured GPU path

    threads = max(1, min(16, os.cpu_count() or 1))
    t0 = time.perf_counter()
    r1, _ = oracle.run_batch(scn, 0, 1, threads=1)
    one = max(time.perf_counter() - t0, 1e-4)
    n = int(max(threads, min(scn.n_replicas, seconds * threads / one)))
    t0 = time.perf_counter()
    res, hashes = oracle.run_batch(scn, 0, n, threads=threads)
    dt = time.perf_counter() - t0
    ev = int(res["events"].sum())
    parity = all(np.array_equal(res[f], gpu_res[f][:n]) for f in res.dtype.names) and \
        np.array_equal(hashes, gpu_hashes[:n])
    return {
        "value": ev / dt, "unit": "events/s", "cores": threads, "kind": "port",
        "sample": f"replicas [0,{n}) of the same workload, oracle canonical mode, {threads} std::threads, "
                  f"{ev} events in {dt:.2f} s",
    }, parity, n


def bench_gossip(args, scn, workload, world, rank, local, dist_on, barrier):
    """Config 4: ONE scenario partitioned by node over the GPUs (strong scaling)."""
    import torch

    from timewarp import dist as twd
    from timewarp.engine import LPEngine, lp_scenario

    L = int(scn.meta["lookahead_us"])
    N = scn.n_nodes
    b0, b1 = twd.strong_block(N, world, rank)
    starts = np.array([twd.strong_block(N, world, r)[0] for r in range(world)])
    dev = f"cuda:{local}" if dist_on else None
    eng = LPEngine(lp_scenario(scn), b0, b1 - b0, L, local)
    for _ in range(args.warmup):
        eng.reset()
        twd.lp_loop(eng, starts, L, dev, dist_on)
    elapsed, kms, windows = 0.0, 0.0, 0
    for _ in range(args.steps):
        eng.reset()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        w, k = twd.lp_loop(eng, starts, L, dev, dist_on)
        torch.cuda.synchronize()
        barrier()
        elapsed += time.perf_counter() - t0
        kms += k
        windows = w
    agg, h = eng.lp_results()
    if dist_on:
        tot, hashes = twd.reduce_lp(agg, h, dev)
        (max_elapsed,) = [twd.reduce_stats({"elapsed_s": elapsed}, device=dev)["elapsed_s"]]
    else:
        tot, hashes, max_elapsed = {f: int(agg[f]) for f in agg.dtype.names}, h, elapsed
    if rank == 0:
        ev = int(tot["events"])
        sends = int(tot["delivered"]) + int(tot["dropped"]) + int(tot["undeliverable"])
        achieved = (64 * ev + 8 * sends) / max(kms / args.steps / 1e3, 1e-12) / 1e9
        out = {
            "metric": "committed events/sec (whole node), gossip 1M nodes node-partitioned",
            "value": ev * args.steps / max_elapsed, "unit": "events/s", "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": max_elapsed * 1e3 / args.steps, "higher_is_better": True,
            "scaling": "strong", "vs_baseline": None, "dtype": "int64",
            "data": "synthetic (peers and link delays drawn from random-1.1 StdGen)",
            "config": {"workload": workload, "nodes": N, "events_per_step": ev, "windows": windows,
                       "parallelism": f"node-partitioned x{world}, RCCL all-to-all per window"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None, "kernel": "tw_run_kernel<LP>",
                         "kernel_ms_per_step": kms / args.steps},
        }
        if not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle

            t0 = time.perf_counter()
            o = oracle.run(scn, trace_cap=0)
            dt = time.perf_counter() - t0
            out["cpu_baseline"] = {"value": o.result["events"] / dt, "unit": "events/s", "cores": 1, "kind": "port",
                                   "sample": f"the whole scenario, sequential oracle (canonical), {dt:.1f} s"}
            out["parity_sample"] = {"scenario": "whole", "bit_exact": bool(
                all(int(tot[f]) == int(o.result[f]) for f in ("final_t", "events", "delivered", "dropped", "undeliverable", "threads"))
                and np.array_equal(hashes, o.hashes))}
        print(json.dumps(out), flush=True)
    eng.close()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="token_ring", choices=["token_ring", "ping_pong", "hotspot", "gossip"])
    ap.add_argument("--replicas", type=int, default=None,
                    help="replicas per GPU: 65536 (token_ring, C3), 1048576 (ping_pong, C2), 4096 (hotspot, C5)")
    ap.add_argument("--nodes", type=int, default=None, help="4096 (token_ring), 256 senders (hotspot), 1M (gossip)")
    ap.add_argument("--duration-s", type=int, default=120)
    ap.add_argument("--drop-log2", type=int, default=10)
    ap.add_argument("--round-trips", type=int, default=1000)
    ap.add_argument("--msg-num", type=int, default=1000)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    args = ap.parse_args()
    if args.nodes is None:
        args.nodes = {"token_ring": 4096, "hotspot": 256, "gossip": 1 << 20}.get(args.config, 2)
    if args.replicas is None:
        args.replicas = {"token_ring": 65536, "ping_pong": 1 << 20, "hotspot": 4096}.get(args.config, 1)

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))

    import torch
    import torch.distributed as dist

    dist_on = world > 1
    if dist_on:
        torch.cuda.set_device(local)
        dist.init_process_group("nccl")

    def barrier():
        if dist_on:
            dist.barrier()

    from timewarp import dist as twd
    from timewarp.engine import Engine

    scn, workload = build_scenario(args, rank)
    if args.config == "gossip":
        return bench_gossip(args, scn, workload, world, rank, local, dist_on, barrier)
    eng = Engine(local).load(scn)

    for _ in range(args.warmup):
        eng.reset()
        eng.run()

    elapsed = 0.0
    events = sends = 0
    kernel_ms = 0.0
    launches = 0
    for _ in range(args.steps):
        eng.reset()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        st = eng.run()
        torch.cuda.synchronize()
        barrier()
        elapsed += time.perf_counter() - t0
        events += st.events
        sends += st.sends
        print(f"[bench] rank {rank} step: {st.events} events in {(time.perf_counter() - t0) * 1e3:.1f} ms",
              file=sys.stderr, flush=True)
        kernel_ms += float(eng.launch_ms().sum())
        launches += st.launches
        if st.replicas_error:
            raise SystemExit(f"{st.replicas_error} replicas ended in an error status")

    res = eng.results()
    hashes = eng.hashes()
    tot = twd.reduce_stats({"events": events, "sends": sends, "elapsed_s": elapsed},
                           device=f"cuda:{local}" if dist_on else None)
    tot_events, max_elapsed = tot["events"], tot["elapsed_s"]

    if rank == 0:
        value = tot_events / max_elapsed
        alg_bytes = BYTES_PER_EVENT * events + BYTES_PER_SEND * sends   # this rank, K steps
        achieved = alg_bytes / (kernel_ms / 1e3) / 1e9 if kernel_ms > 0 else 0.0
        out = {
            "metric": "committed events/sec (whole node) + % HBM roofline, token-ring 64k replicas"
            if args.config == "token_ring" else f"committed events/sec (whole node), {args.config}",
            "value": value,
            "unit": "events/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": max_elapsed * 1e3 / args.steps,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "int64",
            "data": "synthetic (scenario tables drawn from random-1.1 StdGen, seed = replica id)",
            "config": {
                "workload": workload,
                "replicas_per_gpu": args.replicas,
                "events_per_step": int(tot_events / args.steps),
                "parallelism": f"replica-sharded x{world} (no data-path collective)",
            },
            "roofline": {
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": achieved / HBM_PEAK_GBS,
                "traffic": None,
                "kernel": "tw_run_kernel",
                "launches": launches,
                "avg_launch_ms": kernel_ms / max(1, launches),
                "algorithmic_bytes": "64 B/event + 8 B/send (SURVEY.md 8d)",
            },
        }
        prof = os.path.join(ROOT, "profiles", "pmc_summary.json")
        if os.path.exists(prof) and args.config == "token_ring" and args.replicas == 65536 and args.nodes == 4096:
            # measured HBM bytes of the same workload (tools/pmc.sh: separate --pmc passes over a 1-step run
            # of this bench), per launch like `achieved`: one step's traffic / one step's launches
            pm = json.load(open(prof))
            if pm.get("bench_args", "").strip() == "" and "hbm_bytes_total" in pm:
                per_step = float(pm["hbm_bytes_total"])
                out["roofline"]["traffic"] = per_step / max(1, launches / args.steps)
                out["roofline"]["traffic_unit"] = ("HBM bytes per launch: rocprofv3 (2*FETCH_SIZE + WRITE_SIZE)*1024 "
                                                   "over one step's tw_run_kernel dispatches / its launches "
                                                   "(profiles/pmc_summary.json, MI355X_MICROARCH.md HBM section)")
                out["roofline"]["traffic_per_event"] = per_step / max(1, events / args.steps)
                out["roofline"]["algorithmic_per_event"] = alg_bytes / max(1, events)
        if not args.no_cpu_baseline:
            cb, parity, n = cpu_baseline(scn, res, hashes, args.cpu_seconds)
            out["cpu_baseline"] = cb
            out["parity_sample"] = {"replicas": n, "bit_exact": bool(parity)}
        print(json.dumps(out), flush=True)
    eng.close()
    if dist_on:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
