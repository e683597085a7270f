"""Replica sharding across GPUs (one process per GPU, torch.distributed).

Replicas are independent runTimedT calls, so the only cross-GPU traffic is the
statistics reduction (RCCL all-reduce over xGMI with the "nccl" backend, or
gloo on CPU): there is no data-path collective.

Weak scaling (the default of bench.py): rank g owns the global replicas
[g*R, (g+1)*R) and draws their link tables from mkStdGen(g*R + i), so the
union over ranks is bit-identical to one process running all world*R replicas.
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
