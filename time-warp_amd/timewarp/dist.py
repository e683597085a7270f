"""Replica sharding across GPUs (one process per GPU, torch.distributed).

Replicas are independent runTimedT calls, so the only cross-GPU traffic is the
statistics reduction: there is no data-path collective.  The collectives of
the product path belong to the library (include/timewarp.h tw_create_rank):
`library_comm` only hands rank 0's RCCL job id to every rank; tw_run then
all-reduces its statistics and tw_lp_run exchanges a node-partitioned
scenario's records over the library's own RCCL communicator.  The
torch.distributed helpers below remain the thin caller-side pieces (the
barrier and elapsed-time max of bench.py) and the caller-driven window loops,
which the gloo tests exercise on CPU.

Strong scaling (bench.py's default, BASELINE config 3: "64k replicas
sharded across 1/2/4/8 GPUs"): one batch of R replicas is split into
contiguous blocks, rank g owning [g*R/G, (g+1)*R/G) (strong_block).  Weak
scaling (`bench.py --weak`, and the token ring's `weak_line` beside the
strong line at N > 1): every rank runs R replicas of its own, global ids
[g*R, (g+1)*R) (weak_block).  Either way a rank draws its link tables from
mkStdGen(global replica id), so the union over ranks is bit-identical to one
process running all of them.
"""
from __future__ import annotations

from typing import Dict, Tuple

import numpy as np

SUM_KEYS = ("events", "sends", "delivered", "dropped", "undeliverable", "replicas_done", "replicas_error")
MAX_KEYS = ("max_final_t", "elapsed_s", "kernel_ms")


def weak_block(rank: int, replicas_per_rank: int) -> Tuple[int, int]:
    """(seed_base, n_replicas) of this rank's block."""
    return rank * replicas_per_rank, replicas_per_rank


def strong_block(total: int, world: int, rank: int) -> Tuple[int, int]:
    """Contiguous [r0, r1) split of `total` replicas over `world` ranks."""
    base, rem = divmod(total, world)
    r0 = rank * base + min(rank, rem)
    return r0, r0 + base + (1 if rank < rem else 0)


def library_comm(world: int, rank: int):
    """(nranks, rank, job id) for Engine(comm=...): rank 0 makes the RCCL job
    id (tw_comm_id) and torch.distributed broadcasts it; the library then
    creates and owns the communicator (ncclCommInitRank)."""
    import torch.distributed as dist

    from .engine import comm_id

    box = [comm_id() if rank == 0 else None]
    dist.broadcast_object_list(box, src=0)
    return world, rank, box[0]


def reduce_stats(local: Dict[str, float], device=None) -> Dict[str, float]:
    """All-reduce per-rank run statistics: sums of counters, max of times."""
    import torch
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return dict(local)
    s = torch.tensor([float(local.get(k, 0)) for k in SUM_KEYS], dtype=torch.float64, device=device)
    m = torch.tensor([float(local.get(k, 0)) for k in MAX_KEYS], dtype=torch.float64, device=device)
    dist.all_reduce(s, op=dist.ReduceOp.SUM)
    dist.all_reduce(m, op=dist.ReduceOp.MAX)
    out = dict(local)
    out.update({k: v for k, v in zip(SUM_KEYS, s.tolist())})
    out.update({k: v for k, v in zip(MAX_KEYS, m.tolist())})
    return out


def gather_results(res: np.ndarray, hashes: np.ndarray):
    """All-gather per-replica results and hashes (rank order = global replica order)."""
    import torch.distributed as dist

    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return res, hashes
    objs = [None] * dist.get_world_size()
    dist.all_gather_object(objs, (res, hashes))
    return np.concatenate([o[0] for o in objs]), np.concatenate([o[1] for o in objs])


# ------------------------------------------------------ node-partitioned (C4)
INT64_MAX = (1 << 63) - 1


def exchange_records(recs: np.ndarray, owner: np.ndarray, device=None) -> np.ndarray:
    """All-to-all of delivery records (tw_lp_record, 32 B each) to their owning
    ranks: counts first, then the payload with uneven splits.  Over the "nccl"
    backend this is RCCL's all-to-all on xGMI; over gloo it runs on CPU."""
    import torch
    import torch.distributed as dist

    from .engine import LP_RECORD_DTYPE

    world = dist.get_world_size()
    order = np.argsort(owner, kind="stable")
    recs = np.ascontiguousarray(recs[order])
    send_counts = np.bincount(owner, minlength=world).astype(np.int64)
    sc = torch.from_numpy(send_counts).to(device) if device else torch.from_numpy(send_counts)
    rc = torch.empty_like(sc)
    dist.all_to_all_single(rc, sc)
    recv_counts = rc.cpu().numpy()
    raw = recs.view(np.uint8).reshape(-1)
    send_t = torch.from_numpy(raw.copy())
    if device:
        send_t = send_t.to(device)
    recv_t = torch.empty(int(recv_counts.sum()) * LP_RECORD_DTYPE.itemsize, dtype=torch.uint8,
                         device=send_t.device)
    dist.all_to_all_single(recv_t, send_t,
                           output_split_sizes=(recv_counts * LP_RECORD_DTYPE.itemsize).tolist(),
                           input_split_sizes=(send_counts * LP_RECORD_DTYPE.itemsize).tolist())
    return recv_t.cpu().numpy().view(LP_RECORD_DTYPE).copy()


def allreduce_min(v: int, device=None) -> int:
    import torch
    import torch.distributed as dist

    t = torch.tensor([v], dtype=torch.int64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MIN)
    return int(t.item())


def reduce_lp(agg, hashes: np.ndarray, device=None):
    """Sum counters / max times / sum node hashes (mod 2^64) over ranks."""
    import torch
    import torch.distributed as dist

    sums = torch.tensor([int(agg[f]) for f in ("events", "delivered", "dropped", "undeliverable", "threads")],
                        dtype=torch.int64, device=device)
    maxs = torch.tensor([int(agg[f]) for f in ("final_t", "status", "main_exc")], dtype=torch.int64, device=device)
    h = torch.from_numpy(hashes.view(np.int64).copy())
    if device:
        h = h.to(device)
    dist.all_reduce(sums, op=dist.ReduceOp.SUM)
    dist.all_reduce(maxs, op=dist.ReduceOp.MAX)
    dist.all_reduce(h, op=dist.ReduceOp.SUM)  # two's-complement wrap == sum mod 2^64
    out = dict(zip(("events", "delivered", "dropped", "undeliverable", "threads"), sums.tolist()))
    out.update(zip(("final_t", "status", "main_exc"), maxs.tolist()))
    return out, h.cpu().numpy().view(np.uint64).copy()


def lp_loop(eng, starts: np.ndarray, lookahead_us: int, device=None, distributed: bool = True,
            max_windows: int = 1 << 20):
    """Conservative window loop of one rank's LPEngine; returns (windows, kernel_ms)."""
    from .engine import LP_RECORD_DTYPE

    T, windows, kms = 0, 0, 0.0
    while T < INT64_MAX and windows < max_windows:
        nt, nf = eng.window(T + lookahead_us)
        kms += float(eng.launch_ms().sum())
        out = eng.take_outbox() if nf else np.zeros(0, LP_RECORD_DTYPE)
        if distributed:
            owner = np.searchsorted(starts, out["dst"], side="right") - 1
            inc = exchange_records(out, owner.astype(np.int64), device)
            if inc.size:
                nt = min(nt, eng.inject(inc))
            T = allreduce_min(nt, device)
        else:
            if out.size:
                nt = min(nt, eng.inject(out))
            T = nt
        windows += 1
    return windows, kms


def lp_loop_device(eng, world: int, rank: int, starts: np.ndarray, device=None, cap: int = 1 << 14,
                   check_every: int = 16, max_ticks: int = 1 << 22):
    """The device-driven window loop of one rank (tw_lp_tick ...): per tick the
    event kernel + local delivery + packing, an all-to-all of fixed-size record
    blocks, the import, an all-reduce(min) of {next time, -active lanes}, and
    the device-side advance.  The reduction words are {next time, -active
    lanes, -overflow bits}, so an overflow on one rank stops every rank at the
    same tick.  The host enqueues `check_every` ticks between
    synchronisations (tw_lp_progress); no record ever goes through host memory.
    `starts` has world + 1 entries.  Over the "nccl" backend the collectives
    are RCCL on xGMI on the same stream as the engine's kernels.  `cap`
    records per destination rank per tick (the all-to-all moves
    world * (cap + 1) * 32 bytes per rank per tick; C4 at 1M nodes over 8 GPUs
    sends ~1.5k per pair per window); an overflow is an error, never a loss.
    Returns the final tw_lp_state."""
    import torch

    starts = np.asarray(starts, dtype=np.uint32)
    if world == 1:
        eng.exchange_setup(1, 0, starts)  # the context's own stream; run_windows synchronises it
        eng.loop_begin()
        return eng.run_windows(max_ticks)
    bufs = lp_loop_device_setup(eng, world, rank, starts, device, cap)
    with torch.cuda.stream(bufs["stream"]):
        return _lp_ticks(eng, rank, bufs["send"], bufs["recv"], bufs["red"], check_every, max_ticks)


def lp_loop_device_setup(eng, world: int, rank: int, starts: np.ndarray, device=None, cap: int = 1 << 14):
    """The exchange buffers, the boundary table and the stream the engine and
    the collectives share (one ordered, non-default stream) for
    lp_loop_device: made once per engine and kept on it, so later runs (and
    bench.py's timed steps) are the window loop only."""
    import torch

    starts = np.asarray(starts, dtype=np.uint32)
    key = (world, rank, cap, tuple(starts.tolist()))
    bufs = getattr(eng, "_loop_bufs", None)
    if bufs is None or bufs["key"] != key:
        stream = torch.cuda.Stream(device) if device is not None else None
        blk = (cap + 1) * 32
        with torch.cuda.stream(stream):
            send = torch.zeros(world * blk, dtype=torch.uint8, device=device)
            recv = torch.zeros_like(send)
            red = torch.zeros(4, dtype=torch.int64, device=device)
            eng.exchange_tensors(world, rank, starts, send, recv, cap, red)
        if stream is not None:
            stream.synchronize()
        bufs = eng._loop_bufs = dict(key=key, stream=stream, send=send, recv=recv, red=red)
    return bufs


def _lp_ticks(eng, rank, send, recv, red, check_every, max_ticks):
    import torch.distributed as dist

    eng.loop_begin()
    ticks, st = 0, None
    while ticks < max_ticks:
        for _ in range(check_every):
            eng.tick()
            dist.all_to_all_single(recv, send)   # equal splits: block g -> rank g
            eng.tick_import()
            dist.all_reduce(red, op=dist.ReduceOp.MIN)
            eng.tick_end()
        ticks += check_every
        st = eng.progress()
        if st.err:
            # the overflow bits travel in the third reduction word, so every
            # rank stops at the same tick and raises here together (bit 16:
            # stopped because another rank overflowed)
            raise RuntimeError(f"device window loop: overflow bits {st.err} on rank {rank}")
        if st.done:
            break
    return st


def run_partitioned_dist(scn, lookahead_us=None, device_index: int = 0, max_windows: int = 1 << 20):
    """One scenario partitioned by node over all ranks (one GPU each):
    conservative windows [T, T+L), records exchanged by all-to-all, next T by
    an all-reduce(min) of the ranks' next-event times (GVT)."""
    import torch.distributed as dist

    from .engine import LPEngine, lp_scenario

    L = int(lookahead_us if lookahead_us is not None else scn.meta["lookahead_us"])
    world, rank = dist.get_world_size(), dist.get_rank()
    N = scn.n_nodes
    b0, b1 = strong_block(N, world, rank)
    starts = np.array([strong_block(N, world, r)[0] for r in range(world)])
    dev = f"cuda:{device_index}" if dist.get_backend() == "nccl" else None
    eng = LPEngine(lp_scenario(scn), b0, b1 - b0, L, device_index)
    try:
        windows, _ = lp_loop(eng, starts, L, dev, True, max_windows)
        agg, h = eng.lp_results()
        tot, hashes = reduce_lp(agg, h, dev)
        return tot, hashes, windows
    finally:
        eng.close()
