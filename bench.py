#!/usr/bin/env python3
"""Benchmark: committed events/s of the batched TimedT emulator (+ % HBM roofline).

Default workload = BASELINE.json config 3: token-ring, 4096 nodes, 65,536
replicas per GPU, network delay U[1 ms, 5 ms], drop 2^-10 per send
(examples/token-ring/Main.hs lowered).  One "step" = reset every
replica on the device-resident tables and run all of them to quiescence
(runTimedT, src/Control/TimeWarp/Timed/TimedT.hs:293-304).  An event = one
PQ.minView pop of the TimedT schedule (TimedT.hs:242); the GPU count equals the
oracle's (parity-checked on a sample each run).

Multi-GPU: one process per GPU (torchrun).  The replica configs shard
independent replicas over the ranks with no data-path collective (only the
statistics are all-reduced over RCCL).  By default ONE batch of `--replicas`
is split into contiguous blocks [g*R/G, (g+1)*R/G) -- BASELINE config 3, "64k
replicas sharded across 1/2/4/8 GPUs" (8,192 per GPU at 8, where a replica's
own ~45.7k-event chain bounds the step) -- and for the token
ring at N > 1 the weak figure (every rank a 64k batch of its own, seeds
[g*R, (g+1)*R)) is measured after it and reported beside it as `weak_line`.
`--weak` makes the weak split the line itself.  C4 (gossip) partitions one
scenario by node (strong scaling, RCCL all-to-all per window).
"""
from __future__ import annotations

import argparse
import functools
import hashlib
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "time-warp_amd"))

import numpy as np  # noqa: E402

TABLE_CHECK_REPLICAS = 64     # replicas of a device-drawn link table re-drawn on the host
HBM_PEAK_GBS = 8000.0           # MI355X HBM3E peak (MI355X_MICROARCH.md)
BYTES_PER_EVENT = 64            # 16 B event read + 16 B event write + 32 B thread/node state r/w
BYTES_PER_SEND = 8              # link-table entry + ordinal


def replica_block(args, rank: int, world: int):
    """(seed_base, n_replicas) of this rank: `--replicas` of its own (weak
    scaling, the default) or a contiguous block of one batch (`--strong`)."""
    from timewarp.dist import strong_block, weak_block

    if args.weak:
        return weak_block(rank, args.replicas)
    r0, r1 = strong_block(args.replicas, world, rank)
    return r0, r1 - r0


def build_scenario(args, rank: int, world: int, drawer=None, max_replicas=None):
    """This rank's scenario; `drawer` = engine.draw_link_table draws its link
    table on the GPU (tw_draw_link_table) instead of the host StdGen loop;
    `max_replicas` caps the block (the host-drawn table check)."""
    from timewarp import scenarios

    base, R = replica_block(args, rank, world)
    if max_replicas is not None:
        R = min(R, max_replicas)
    per = "/GPU" if args.weak else "" if world == 1 else f" (rank {rank} of {world}: [{base}, {base + R}) of {args.replicas})"
    if args.config == "token_ring":
        return scenarios.token_ring(n_nodes=args.nodes, n_replicas=R, launch_duration=args.duration_s * 1_000_000,
                                    drop_log2=args.drop_log2, seed_base=base, drawer=drawer), (
            f"token-ring (examples/token-ring) {args.nodes} nodes x {R} replicas{per}, delay U[1,5] ms, "
            f"drop 2^-{args.drop_log2}, launchDuration {args.duration_s} s")
    if args.config == "ping_pong":
        return scenarios.ping_pong(n_replicas=R, round_trips=args.round_trips, seed_base=base, drawer=drawer), (
            f"ping-pong (examples/ping-pong) 2 nodes x {R} replicas{per}, {args.round_trips} round trips, "
            "per-link delay U[1,5] ms")
    if args.config == "hotspot":
        return scenarios.hotspot(n_senders=args.nodes, n_replicas=R, msg_num=args.msg_num, seed_base=base,
                                 drawer=drawer), (
            f"hotspot (bench/Network) {args.nodes} senders -> 1 receiver x {R} replicas{per}, "
            f"{args.msg_num} msgs @1000/s")
    if args.config == "gossip":
        return scenarios.gossip(n_nodes=args.nodes, seed=0), (
            f"gossip (config 4) one scenario of {args.nodes} nodes, fanout 4, delay U[1,5] ms, "
            f"node-partitioned over the GPUs, lookahead 1 ms windows")
    raise SystemExit(f"unknown config {args.config}")


def host_cpu():
    """(threads, description): `nproc` (the CPUs this process may use; honours
    affinity and OMP_NUM_THREADS, 16 on the GPU box) and the CPU model."""
    try:
        n = int(subprocess.run(["nproc"], capture_output=True, text=True, check=True).stdout.strip())
    except Exception:
        n = len(os.sched_getaffinity(0)) if hasattr(os, "sched_getaffinity") else (os.cpu_count() or 1)
    model = "unknown"
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                model = line.split(":", 1)[1].strip()
                break
    except OSError:
        pass
    return max(1, n), f"{model}; nproc {n} of {os.cpu_count()} logical CPUs"


def cpu_baseline(scn, gpu_res, gpu_hashes, seconds: float):
    """Oracle (C++ TimedT restatement, canonical mode) on host cores, bounded
    sample; one replica per std::thread worker, a pool of `nproc` workers
    (SURVEY.md 8(d))."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # the parity checker / CPU baseline — never the measured GPU path

    threads, cpu_desc = host_cpu()
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
        "value": ev / dt, "unit": "events/s", "cores": threads, "kind": "port", "cpu": cpu_desc,
        "sample": f"replicas [0,{n}) of the same workload, oracle canonical mode, {threads} std::threads "
                  f"(nproc), {ev} events in {dt:.2f} s; the reference TimedT itself cannot run here (no GHC, "
                  f"so no RTS -N)",
    }, parity, n


def engine_sha() -> str:
    """Digest of the engine sources: a PMC summary is used only for the build it measured."""
    h = hashlib.sha256()
    d = os.path.join(ROOT, "time-warp_amd", "csrc")
    for f in sorted(os.listdir(d)):
        h.update(f.encode())
        h.update(open(os.path.join(d, f), "rb").read())
    return h.hexdigest()[:16]


def measured_traffic(args, launches_per_step: float, events_per_step: float, whole_loop: bool = False):
    """HBM traffic of this workload from the newest profiles/*/pmc_summary.json
    taken with tools/pmc.sh on THIS engine build (engine_sha) and the same
    workload (bench_workload); None otherwise.  rocprofv3 PMC counters cannot
    be read inside the un-profiled timed run itself."""
    want = workload_key(args)
    best = None
    for root, _, files in os.walk(os.path.join(ROOT, "profiles")):
        if "pmc_summary.json" not in files:
            continue
        f = os.path.join(root, "pmc_summary.json")
        try:
            pm = json.load(open(f))
        except (OSError, ValueError):
            continue
        if pm.get("engine_sha") != engine_sha() or pm.get("bench_workload") != want or "fetch_size" not in pm:
            continue
        if best is None or f > best[0]:
            best = (f, pm)
    if best is None:
        return None
    f, pm = best
    key = "hbm_bytes_all_tw" if whole_loop else "hbm_bytes_total"
    if key not in pm:
        return None
    per_step = float(pm[key]) / max(1, int(pm.get("steps", 1)))
    return {
        "traffic": per_step / max(1.0, launches_per_step),
        "traffic_per_event": per_step / max(1.0, events_per_step),
        "fetch_size_kib": pm["fetch_size_all_tw" if whole_loop else "fetch_size"],
        "write_size_kib": pm["write_size_all_tw" if whole_loop else "write_size"],
        "traffic_scope": "every kernel of the window loop (one launch = the loop)" if whole_loop else
                         "the event kernel, per launch",
        "traffic_formula": pm.get("formula", "(2*FETCH_SIZE + WRITE_SIZE)*1024"),
        "traffic_source": os.path.relpath(f, ROOT) + f" (engine {pm['engine_sha']})",
    }


def workload_key(args) -> str:
    return (f"{args.config}:nodes={args.nodes}:replicas={args.replicas}:weak={int(args.weak)}:"
            f"dur={args.duration_s}:drop={args.drop_log2}:rt={args.round_trips}:msgs={args.msg_num}"
            + (f":geo={args.geometry}" if getattr(args, "geometry", None) else "")
            + (f":tie={args.tie}" if getattr(args, "tie", "auto") != "auto" else ""))


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
    # one rank of the job: the library owns the RCCL communicator over the
    # ranks (tw_create_rank); its window loop (tw_lp_run) exchanges record
    # blocks and reduces the window words itself, and tw_lp_results is the
    # whole job's.  The host-driven loop keeps per-rank contexts.
    comm = twd.library_comm(world, rank) if dist_on and not args.host_windows else None
    eng = LPEngine(lp_scenario(scn), b0, b1 - b0, L, local, comm=comm)

    def one_run():
        """(windows, ticks, device ms) of one whole-scenario run"""
        if args.host_windows:  # the host-driven loop: tw_lp_window / take_outbox / inject per window
            w, k = twd.lp_loop(eng, starts, L, dev, dist_on)
            return w, w, k
        # the device loop synchronises its stream before returning, so the
        # wall time of the call is the loop's device time (+ one sync); its
        # exchange buffers are made by the first (warm-up) run
        t0 = time.perf_counter()
        st = eng.run_lp()
        return int(st.windows), int(st.ticks), (time.perf_counter() - t0) * 1e3

    for _ in range(args.warmup):
        eng.reset()
        one_run()
    elapsed, kms, windows, ticks = 0.0, 0.0, 0, 0
    for _ in range(args.steps):
        eng.reset()
        barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        w, tk, k = one_run()
        torch.cuda.synchronize()
        barrier()
        elapsed += time.perf_counter() - t0
        kms += k
        windows, ticks = w, tk
    agg, h = eng.lp_results()
    if int(agg["status"]) >= 2:  # TW_REP_ABORTED or an error status on some node
        raise SystemExit(f"gossip: nodes ended in status {int(agg['status'])}")
    if dist_on and args.host_windows:
        tot, hashes = twd.reduce_lp(agg, h, dev)
    else:  # one context, or the library's job-wide reduction (tw_lp_results)
        tot, hashes = {f: int(agg[f]) for f in agg.dtype.names}, h
    max_elapsed = twd.reduce_stats({"elapsed_s": elapsed}, device=dev)["elapsed_s"] if dist_on else elapsed
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
                       "ticks": ticks,
                       "window_loop": "host (tw_lp_window per window)" if args.host_windows else
                       "device (tw_lp_run: window advance, exchange and GVT on the GPU; one host sync per 16 ticks)",
                       "parallelism": f"node-partitioned x{world}, library-owned RCCL: send/recv of record blocks "
                                      "sized by the ranks' demand + all-reduce(min) of the window words per tick"},
            "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBS, "unit": "GB/s",
                         "frac": achieved / HBM_PEAK_GBS, "traffic": None, "kernel": "tw_run_kernel<LP>",
                         "kernel_ms_per_step": kms / args.steps,
                         "kernel_ms_note": "time of the whole device window loop (event kernels + pack/import/"
                                           "advance kernels + collectives), up to its final stream sync"
                         if not args.host_windows else "summed event-kernel launches"},
        }
        mt = measured_traffic(args, 1, ev, whole_loop=True) if world == 1 and not args.host_windows else None
        if mt:
            out["roofline"].update(mt)
        if not args.no_cpu_baseline:
            sys.path.insert(0, os.path.join(ROOT, "oracle"))
            import oracle

            t0 = time.perf_counter()
            o = oracle.run(scn, trace_cap=0)
            dt = time.perf_counter() - t0
            threads, cpu_desc = host_cpu()
            if world == 1:  # (the CPU baseline: rank 0 at N=1 only; at N > 1 the run is the parity check)
                out["cpu_baseline"] = {
                    "value": o.result["events"] / dt, "unit": "events/s", "cores": 1, "kind": "port", "cpu": cpu_desc,
                    "sample": f"the whole scenario, sequential oracle (canonical), {dt:.1f} s; one "
                              f"thread by design, not the {threads} of nproc: C4 is ONE scenario, and "
                              f"TimedT runs a scenario as one sequential loop (TimedT.hs:239-263)"}
            out["parity_sample"] = {"scenario": "whole", "bit_exact": bool(
                all(int(tot[f]) == int(o.result[f]) for f in ("final_t", "events", "delivered", "dropped", "undeliverable", "threads"))
                and np.array_equal(hashes, o.hashes))}
        print(json.dumps(out), flush=True)
    eng.close()


def pick_geometry(args, world):
    """The default kernel geometry of a replica config for this rank's share."""
    if args.geometry is None and args.config == "hotspot":
        # C5: a replica is one long chain in the replica geometries (0.32 G
        # events/s, wave); its nodes as logical processes run it in parallel
        args.geometry = "lpb"
    if args.geometry is None and args.config == "token_ring":
        # C3 split 8 ways (8,192 replicas per GPU): a replica's ~45.7k-event
        # chain bounds the replica geometries (narrow 2.5 G events/s); its
        # (node, replica) pairs as logical processes run it at 3.6 G.  From
        # 16,384 replicas per GPU up, narrow/dense win (5.3 vs 4.2 G at 16k).
        per = args.replicas if args.weak else args.replicas // max(world, 1)
        if per <= 8192 and per & (per - 1) == 0 and args.replicas % max(world, 1) == 0:
            args.geometry = "lpb"


def parity_sample(scn, gpu_res, gpu_hashes, seconds: float):
    """(bit_exact, n): the oracle on replicas [0, n) of this rank's batch,
    about `seconds` of host work (N > 1: no CPU baseline is timed, but every
    run still checks a sample of its own replicas)."""
    sys.path.insert(0, os.path.join(ROOT, "oracle"))
    import oracle  # the parity checker -- never the measured GPU path

    threads, _ = host_cpu()
    t0 = time.perf_counter()
    oracle.run_batch(scn, 0, 1, threads=1)
    one = max(time.perf_counter() - t0, 1e-4)
    n = int(max(1, min(scn.n_replicas, seconds * threads / one)))
    res, hashes = oracle.run_batch(scn, 0, n, threads=threads)
    ok = all(np.array_equal(res[f], gpu_res[f][:n]) for f in res.dtype.names) and \
        np.array_equal(hashes, gpu_hashes[:n])
    return ok, n


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=1)
    ap.add_argument("--config", default="token_ring", choices=["token_ring", "ping_pong", "hotspot", "gossip"])
    ap.add_argument("--replicas", type=int, default=None,
                    help="replicas of the job: 65536 (token_ring, C3), 1048576 (ping_pong, C2), 4096 (hotspot, "
                         "C5), split over the GPUs (BASELINE config 3: 64k replicas sharded across 1/2/4/8 GPUs); "
                         "with --weak, per GPU")
    ap.add_argument("--strong", action="store_true", help="(the default: one batch of --replicas split over the GPUs)")
    ap.add_argument("--weak", action="store_true",
                    help="--replicas per GPU (weak scaling) instead of one batch split over the GPUs")
    ap.add_argument("--no-weak-line", action="store_true",
                    help="token_ring at N > 1: skip the weak-scaling figure (a 64k batch per GPU) that is "
                         "measured after the strong split and reported beside it as weak_line")
    ap.add_argument("--nodes", type=int, default=None, help="4096 (token_ring), 256 senders (hotspot), 1M (gossip)")
    ap.add_argument("--duration-s", type=int, default=120)
    ap.add_argument("--drop-log2", type=int, default=10)
    ap.add_argument("--round-trips", type=int, default=1000)
    ap.add_argument("--msg-num", type=int, default=1000)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--host-tables", action="store_true",
                    help="draw the link tables with the host StdGen loop instead of on the GPU")
    ap.add_argument("--geometry", default=None, choices=["dense", "sparse", "half", "wave", "narrow", "compact", "lpb"],
                    help="replica configs: kernel geometry (default: the library's choice by replica count); "
                         "lpb = every (node, replica) a logical process in one window loop (the replicas per "
                         "GPU must be a power of two: lanes are node << log2(R) | replica)")
    ap.add_argument("--host-windows", action="store_true",
                    help="gossip: the host-driven window loop (round-1 path) instead of the device loop")
    ap.add_argument("--tie", default="auto", choices=["auto", "fifo", "forkfirst", "lifo"],
                    help="equal-timestamp order (tw_set_tie_mode).  forkfirst = fifo except that a forked child is "
                         "always the next pop, as in TimedT's pqueue (an insert whose key is <= the held minimum "
                         "becomes the minimum); the replica kernels then run the child in place.  auto: forkfirst "
                         "for the token ring on the lane-per-replica geometries (C3 is tie-insensitive: its results "
                         "equal the canonical order's, checked by parity_sample), else fifo")
    ap.add_argument("--workload-key", action="store_true",
                    help="print the workload key and engine digest (tools/pmc.sh provenance) and exit")
    args = ap.parse_args()
    args.weak = args.weak and not args.strong
    if args.nodes is None:
        args.nodes = {"token_ring": 4096, "hotspot": 256, "gossip": 1 << 20}.get(args.config, 2)
    if args.replicas is None:
        args.replicas = {"token_ring": 65536, "ping_pong": 1 << 20, "hotspot": 4096}.get(args.config, 1)
    args.geometry_auto = args.geometry is None
    pick_geometry(args, int(os.environ.get("WORLD_SIZE", "1")))
    if args.workload_key:
        print(json.dumps({"bench_workload": workload_key(args), "engine_sha": engine_sha()}))
        return

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

    if args.config == "gossip":
        scn, workload, setup = setup_scenario(args, rank, world, local)
        return bench_gossip(args, scn, workload, world, rank, local, dist_on, barrier)
    m = measure_replicas(args, rank, world, local, dist_on, barrier)
    print_line = replica_line(args, world, m) if rank == 0 else None
    # BASELINE config 3 is one 64k batch split over the GPUs (the line above);
    # the weak figure -- every GPU a 64k batch of its own -- is measured after
    # it and sits beside it, never in its place
    if world > 1 and args.config == "token_ring" and not args.weak and not args.no_weak_line:
        wa = argparse.Namespace(**vars(args))
        wa.weak = True
        wa.geometry = None if args.geometry_auto else args.geometry
        pick_geometry(wa, world)
        w = measure_replicas(wa, rank, world, local, dist_on, barrier, parity=False)
        if rank == 0:
            print_line["weak_line"] = {
                "value": w["value"], "ms_per_step": w["ms_per_step"], "scaling": "weak",
                "replicas_per_gpu": w["scn_replicas"], "replicas_total": w["scn_replicas"] * world,
                "geometry": w["geometry"], "tie_order": w["tie"],
                "note": "each GPU its own 65,536-replica batch (seeds [g*R, (g+1)*R)); not BASELINE config 3's "
                        "split, reported beside it"}
    if rank == 0:
        print(json.dumps(print_line), flush=True)
        if "parity_sample" in print_line and not print_line["parity_sample"]["bit_exact"]:
            raise SystemExit("parity_sample: the GPU results differ from the oracle's")
    if dist_on:
        dist.destroy_process_group()


def setup_scenario(args, rank, world, local):
    """This rank's scenario (outside the timed region): the link table drawn on
    the GPU, checked against the host StdGen draw on its first replicas."""
    drawer = None
    if not args.host_tables and args.config != "gossip":
        from timewarp.engine import draw_link_table
        drawer = functools.partial(draw_link_table, device=local)
    t_setup = time.perf_counter()
    scn, workload = build_scenario(args, rank, world, drawer=drawer)
    setup = {"table_draw": "host" if drawer is None else "device (tw_draw_link_table)",
             "build_s": time.perf_counter() - t_setup}
    if drawer is not None and scn.link_table is not None:
        ref, _ = build_scenario(args, rank, world, max_replicas=TABLE_CHECK_REPLICAS)
        n_chk = ref.link_table.shape[2]
        setup["host_check_replicas"] = n_chk
        setup["host_check_equal"] = bool(np.array_equal(scn.link_table[:, :, :n_chk], ref.link_table))
        if not setup["host_check_equal"]:
            raise SystemExit("device-drawn link table differs from the host StdGen draw")
    return scn, workload, setup


def measure_replicas(args, rank, world, local, dist_on, barrier, parity=True):
    """W warm-up and K timed steps of the replica configs on this rank; the
    parity sample (rank 0: the CPU baseline at N = 1, a smaller oracle check of
    its own replicas at N > 1)."""
    import torch

    from timewarp import dist as twd
    from timewarp.engine import Engine

    if args.geometry == "lpb":
        _, r_rank = replica_block(args, rank, world)
        if r_rank & (r_rank - 1):
            raise SystemExit(f"--geometry lpb needs a power-of-two replica count per GPU (lanes are node << log2(R) "
                             f"| replica); rank {rank} of {world} would get {r_rank} of {args.replicas} replicas")
    scn, workload, setup = setup_scenario(args, rank, world, local)
    # one rank of the job: the library's RCCL communicator over the ranks
    # (tw_create_rank) all-reduces every tw_run's statistics
    comm = twd.library_comm(world, rank) if dist_on else None
    eng = Engine(local, comm=comm)
    t_load = time.perf_counter()
    eng.load(scn, geometry=args.geometry)
    setup["load_s"] = time.perf_counter() - t_load
    tie = args.tie
    if tie == "auto":
        tie = "forkfirst" if args.config == "token_ring" and eng.geometry() not in ("lpb", "wave") else "fifo"
    if tie != "fifo":
        eng.set_tie_mode(tie)
    setup["tie_order"] = tie

    for _ in range(args.warmup):
        eng.reset()
        eng.run()

    elapsed = 0.0
    events = sends = 0
    msg = {"delivered": 0, "dropped": 0, "undeliverable": 0}
    kernel_ms = 0.0
    launches = 0
    lpb_wt = None
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
        for k in msg:
            msg[k] += getattr(st, k)
        print(f"[bench] rank {rank} step: {st.events} events in {(time.perf_counter() - t0) * 1e3:.1f} ms",
              file=sys.stderr, flush=True)
        kernel_ms += float(eng.launch_ms().sum())
        launches += st.launches
        if eng.geometry() == "lpb":
            lpb_wt = eng.lpb_windows()
        if st.replicas_error:
            raise SystemExit(f"{st.replicas_error} replicas ended in an error status")

    res = eng.results()
    hashes = eng.hashes()
    # st.* are the job's (tw_run's statistics, all-reduced by the library over
    # the ranks); this rank's own share is in its replicas' results
    m = {"scn_replicas": scn.n_replicas, "workload": workload, "setup": setup, "tie": tie,
         "geometry": eng.geometry(), "lpb_wt": lpb_wt, "steps": args.steps,
         "loc_events": int(res["events"].sum()) * args.steps,
         "loc_sends": int((res["delivered"] + res["dropped"] + res["undeliverable"]).sum()) * args.steps,
         "tot_events": events, "sends": sends, "msg": msg, "kernel_ms": kernel_ms, "launches": launches,
         "threads_forked": int(res["threads"].sum())}
    m["max_elapsed"] = (twd.reduce_stats({"elapsed_s": elapsed}, device=f"cuda:{local}")["elapsed_s"]
                        if dist_on else elapsed)
    m["value"] = events / m["max_elapsed"]
    m["ms_per_step"] = m["max_elapsed"] * 1e3 / args.steps
    eng.close()
    if rank == 0 and parity and not args.no_cpu_baseline:
        if world == 1:  # the CPU baseline: rank 0 at N=1 only; its results double as the parity sample
            cb, ok, n = cpu_baseline(scn, res, hashes, args.cpu_seconds)
            m["cpu_baseline"] = cb
        else:  # N > 1: no CPU timing, but still an oracle check of this rank's own replicas
            ok, n = parity_sample(scn, res, hashes, args.cpu_seconds / 2)
        m["parity_sample"] = {"replicas": n, "bit_exact": bool(ok),
                              "against": "oracle canonical (t, seq) order"
                                         + ("" if world == 1 else f", rank 0's replicas [0,{n}) of its block")}
    return m


def replica_line(args, world, m):
    """The bench JSON line of a replica config from measure_replicas' numbers."""
    value = m["value"]
    alg_bytes = BYTES_PER_EVENT * m["loc_events"] + BYTES_PER_SEND * m["loc_sends"]   # this rank, K steps
    kernel_ms, launches = m["kernel_ms"], m["launches"]
    achieved = alg_bytes / (kernel_ms / 1e3) / 1e9 if kernel_ms > 0 else 0.0
    geometry = m["geometry"]
    out = {
        "metric": "committed events/sec (whole node) + % HBM roofline, token-ring 64k replicas"
        if args.config == "token_ring" else f"committed events/sec (whole node), {args.config}",
        "value": value,
        "unit": "events/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": m["ms_per_step"],
        "higher_is_better": True,
        "scaling": "weak" if args.weak else "strong",
        "vs_baseline": None,
        "dtype": "int64",
        "data": "synthetic (scenario tables drawn from random-1.1 StdGen, seed = replica id)",
        "config": {
            "workload": m["workload"],
            "baseline_config": ("BASELINE config 3: one batch of 65,536 replicas split over the GPUs"
                                if args.config == "token_ring" and not args.weak and args.replicas == 65536 else None),
            "replicas_total": args.replicas * (world if args.weak else 1),
            "replicas_rank0": m["scn_replicas"],
            "events_per_step": int(m["tot_events"] / args.steps),
            "parallelism": (f"replica-sharded x{world}: {m['scn_replicas']} replicas per GPU, seeds [g*R, (g+1)*R) "
                            "(no data-path collective)" if args.weak else
                            f"replica-sharded x{world}: one batch in contiguous blocks (no data-path collective)"),
            "geometry": geometry,
            "tie_order": m["tie"],
        },
        "roofline": {
            "bound": "hbm",
            "achieved": achieved,
            "peak": HBM_PEAK_GBS,
            "unit": "GB/s",
            "frac": achieved / HBM_PEAK_GBS,
            "traffic": None,
            "kernel": "tw_run_kernel" if geometry != "lpb" else "tw_run_kernel<LP> window loop",
            "launches": launches,
            "avg_launch_ms": kernel_ms / max(1, launches),
            "algorithmic_bytes": "64 B/event + 8 B/send (SURVEY.md 8d)",
        },
    }
    out["roofline"]["algorithmic_per_event"] = alg_bytes / max(1, m["loc_events"])
    out["setup"] = m["setup"]
    if geometry == "lpb":
        out["config"]["parallelism"] = (f"replica-sharded x{world}; inside a GPU every (node, replica) pair is a "
                                        "logical process: one device window loop, lookahead = min link delay")
        out["config"]["windows"], out["config"]["ticks"] = m["lpb_wt"]
        out["roofline"]["kernel_ms_note"] = ("one launch = the whole device window loop (event kernels + "
                                             "due/pack/compact/advance kernels), HIP events")
    # what the timed events are (the job, per step): message sends, arrivals
    # (delivered / dropped / no listener), threads forked, and the rest
    # (waits, wake-ups, kills, timeouts)
    per = {k: v // args.steps for k, v in m["msg"].items()}
    per["sends"] = m["sends"] // args.steps
    per["threads_forked"] = m["threads_forked"]
    per["events"] = m["tot_events"] // args.steps
    arrivals = per["delivered"] + per["dropped"] + per["undeliverable"]
    # arrival pops over all pops (each delivered message also forks a
    # handler thread and wakes its receiver: DESIGN.md section 6)
    per["arrivals_frac"] = arrivals / max(1, per["events"])
    out["events_breakdown"] = per
    mt = (measured_traffic(args, launches / args.steps, m["loc_events"] / args.steps, geometry == "lpb")
          if world == 1 else None)
    if mt:
        out["roofline"].update(mt)
    if "cpu_baseline" in m:
        out["cpu_baseline"] = m["cpu_baseline"]
    if "parity_sample" in m:
        out["parity_sample"] = m["parity_sample"]
    return out


if __name__ == "__main__":
    main()
