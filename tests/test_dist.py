"""Multi-rank replica sharding with world_size 2 over gloo (CPU).

Each rank owns a contiguous block of one global batch (strong scaling,
bench.py's default -- BASELINE config 3's 64k over the GPUs: dist.strong_block,
uneven here so the remainder rule is exercised; `bench.py --weak` and the
token ring's weak_line give each rank a batch of its own: dist.weak_block,
test_bench_replica_blocks); the per-rank run (here the oracle, standing in for the per-GPU
engine which needs a device) is reduced with timewarp.dist exactly as bench.py
does over RCCL.  The union must equal a single-process run of all replicas,
replica for replica."""
import os
import socket

import numpy as np
import torch.multiprocessing as mp

R_TOTAL = 25  # split 13 + 12 over two ranks


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, out_path):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "time-warp_amd"), os.path.join(root, "oracle")]
    import torch.distributed as dist

    import oracle
    from timewarp import dist as twd
    from timewarp import scenarios

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    r0, r1 = twd.strong_block(R_TOTAL, world, rank)
    seed_base, n = r0, r1 - r0
    scn = scenarios.token_ring(n_nodes=9, n_replicas=n, launch_duration=30_000_000, drop_log2=3,
                               link_depth=4, seed_base=seed_base)
    res, hashes = oracle.run_batch(scn, threads=2)
    stats = twd.reduce_stats({"events": int(res["events"].sum()), "dropped": int(res["dropped"].sum()),
                              "max_final_t": int(res["final_t"].max()), "elapsed_s": 0.1 * (rank + 1)})
    allres, allh = twd.gather_results(res, hashes)
    if rank == 0:
        np.savez(out_path, res=allres, hashes=allh, events=stats["events"], dropped=stats["dropped"],
                 max_final_t=stats["max_final_t"], elapsed=stats["elapsed_s"])
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_sharding_equals_single_process(tmp_path, oracle_mod):
    from timewarp import dist as twd
    from timewarp import scenarios

    out = str(tmp_path / "r.npz")
    mp.spawn(_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    got = np.load(out)
    scn = scenarios.token_ring(n_nodes=9, n_replicas=R_TOTAL, launch_duration=30_000_000, drop_log2=3,
                               link_depth=4, seed_base=0)
    res, hashes = oracle_mod.run_batch(scn, threads=4)
    for f in res.dtype.names:
        assert np.array_equal(got["res"][f], res[f]), f
    assert np.array_equal(got["hashes"], hashes)
    assert got["events"] == res["events"].sum() and got["dropped"] == res["dropped"].sum()
    assert got["max_final_t"] == res["final_t"].max()
    assert abs(float(got["elapsed"]) - 0.2) < 1e-12  # max over ranks
    assert twd.strong_block(10, 3, 0) == (0, 4) and twd.strong_block(10, 3, 2) == (7, 10)
    assert twd.strong_block(R_TOTAL, 2, 0) == (0, 13) and twd.weak_block(1, 12) == (12, 12)


def _xchg_worker(rank, world, port, out_path):
    import sys

    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path[:0] = [os.path.join(root, "time-warp_amd")]
    import torch.distributed as dist

    from timewarp import dist as twd
    from timewarp.engine import LP_RECORD_DTYPE

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    rng = np.random.default_rng(rank)
    n = 50 + 30 * rank
    recs = np.zeros(n, LP_RECORD_DTYPE)
    recs["t_arr"] = rng.integers(0, 1 << 40, n)
    recs["payload"] = rank * 1000 + np.arange(n)
    recs["dst"] = rng.integers(0, 100, n)
    recs["src"] = rank
    starts = np.array([0, 37])
    owner = np.searchsorted(starts, recs["dst"], side="right") - 1
    got = twd.exchange_records(recs, owner)
    m = twd.allreduce_min(int(recs["t_arr"].min()))
    np.savez(out_path + f".{rank}", got=got, sent=recs, m=m)
    dist.barrier()
    dist.destroy_process_group()


def test_record_exchange_all_to_all(tmp_path):
    """The C4 exchange step (counts + uneven all_to_all_single) over gloo."""
    out = str(tmp_path / "x")
    mp.spawn(_xchg_worker, args=(2, _free_port(), out), nprocs=2, join=True)
    r = [np.load(out + f".{i}.npz") for i in range(2)]
    sent = np.concatenate([r[0]["sent"], r[1]["sent"]])
    starts = np.array([0, 37])
    for rank in range(2):
        owner = np.searchsorted(starts, sent["dst"], side="right") - 1
        exp = np.sort(sent[owner == rank], order=["src", "payload"])
        got = np.sort(r[rank]["got"], order=["src", "payload"])
        assert np.array_equal(exp, got)
        assert int(r[rank]["m"]) == int(sent["t_arr"].min())


def test_bench_replica_blocks():
    """bench.py's rank blocks: --weak (rank g runs global
    replicas [g*R, (g+1)*R), its tables drawn from mkStdGen(g*R + i)), or
    one batch split (the default since round 6: BASELINE config 3's 64k over
    the GPUs); the workload key names the choice, so a PMC summary of one is
    never used for the other.  The default geometry follows the per-GPU share:
    batched logical processes at 8,192 replicas per GPU (8 GPUs), the replica
    kernels from 16,384 up, and the weak line's 64k per GPU."""
    import argparse
    import importlib.util
    import pathlib

    root = pathlib.Path(__file__).resolve().parents[1]
    spec = importlib.util.spec_from_file_location("bench_mod", root / "bench.py")
    bench = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(bench)
    args = argparse.Namespace(replicas=65536, weak=True, config="token_ring", nodes=4096, duration_s=120,
                              drop_log2=10, round_trips=1000, msg_num=1000, geometry=None, tie="auto")
    assert [bench.replica_block(args, g, 8) for g in range(3)] == [(0, 65536), (65536, 65536), (131072, 65536)]
    assert ":weak=1:" in bench.workload_key(args)
    args.weak = False
    blocks = [bench.replica_block(args, g, 8) for g in range(8)]
    assert blocks[0] == (0, 8192) and blocks[7] == (57344, 8192) and sum(n for _, n in blocks) == 65536
    assert ":weak=0:" in bench.workload_key(args)
    for world, geo in ((1, None), (2, None), (4, None), (8, "lpb")):
        a = argparse.Namespace(**vars(args))
        bench.pick_geometry(a, world)
        assert a.geometry == geo, (world, a.geometry)
    a = argparse.Namespace(**vars(args))
    a.weak = True
    bench.pick_geometry(a, 8)
    assert a.geometry is None
