"""timewarp.dist's two window loops for a node-partitioned scenario (config 4)
at world_size 2 over gloo, against a single-process run: the host-driven loop
(dist.lp_loop: tw_lp_window / take_outbox / inject per window, all-to-all of
record lists, all-reduce(min) GVT) and the device-driven loop
(dist.lp_loop_device: tw_lp_tick's fixed record blocks, all-to-all, reduction
words {next time, -active}, advance or rerun).  The per-rank engine is the CPU
stand-in of tests/lp_standin.py (the GPU engine is covered by
tests/test_gpu_gossip.py); what is checked here is the loops and their
collectives: same events, same node hashes, same window count."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

N, L = 60, 1000


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _single(budget):
    from lp_standin import StandinLP
    from timewarp import dist as twd

    e = StandinLP(N, 0, N, L, budget=budget)
    st = twd.lp_loop_device(e, 1, 0, np.array([0, N]))
    ev, h = e.results()
    e2 = StandinLP(N, 0, N, L, budget=budget)
    w2, _ = twd.lp_loop(e2, np.array([0]), L, None, distributed=False)
    assert e2.results()[0] == ev and np.array_equal(e2.results()[1], h)
    assert w2 == st.windows
    return ev, h, st.windows


def _worker(rank, world, port, out_path, mode, budget, overflow_rank=None):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "time-warp_amd"), os.path.join(root, "tests")]
    import torch.distributed as dist

    from lp_standin import StandinLP
    from timewarp import dist as twd

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    b0, b1 = twd.strong_block(N, world, rank)
    starts = np.array([twd.strong_block(N, world, r)[0] for r in range(world)] + [N])
    e = StandinLP(N, b0, b1 - b0, L, budget=budget, overflow_tick=4 if rank == overflow_rank else None)
    if overflow_rank is not None:
        # one rank overflows: both ranks must stop at the same check and raise
        # (the overflow bits are the third reduction word), none left waiting
        # in a collective
        try:
            twd.lp_loop_device(e, world, rank, starts, None, cap=256, check_every=3)
            err = 0
        except RuntimeError as x:
            err = int(str(x).split("overflow bits ")[1].split()[0])
        np.save(f"{out_path}.{rank}.npy", np.array([err, e.ticks]))
        dist.destroy_process_group()
        return
    if mode == "host":
        windows, _ = twd.lp_loop(e, starts[:-1], L, None, distributed=True)
    else:
        windows = twd.lp_loop_device(e, world, rank, starts, None, cap=256, check_every=3).windows
    ev, h = e.results()
    import torch

    t = torch.tensor([ev], dtype=torch.int64)
    dist.all_reduce(t)
    hh = torch.from_numpy(h.view(np.int64).copy())
    dist.all_reduce(hh)
    if rank == 0:
        np.savez(out_path, events=int(t.item()), hashes=hh.numpy().view(np.uint64), windows=windows)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("mode,budget", [("host", 1 << 30), ("device", 1 << 30), ("device", 2)])
def test_two_rank_window_loop_equals_single_process(tmp_path, mode, budget):
    ev, h, windows = _single(budget)
    assert ev > 100 and windows > 5
    out = str(tmp_path / "r.npz")
    mp.spawn(_worker, args=(2, _free_port(), out, mode, budget), nprocs=2, join=True)
    got = np.load(out)
    assert int(got["events"]) == ev
    assert np.array_equal(got["hashes"], h)
    assert int(got["windows"]) == windows


def test_overflow_on_one_rank_stops_both(tmp_path):
    """An inbox overflow on rank 1 only: both ranks' device loops
    stop at the same tick and raise with the overflowing rank's bits (the
    all-reduce(min) of -bits) plus bit 16 (stopped by the shared error word);
    the processes exit."""
    out = str(tmp_path / "o")
    mp.spawn(_worker, args=(2, _free_port(), out, "device", 1 << 30, 1), nprocs=2, join=True)
    e0, t0 = np.load(out + ".0.npy")
    e1, t1 = np.load(out + ".1.npy")
    assert e0 == e1 == 1 | 16
    assert t0 == t1 == 5  # stopped at the tick after the overflow's
