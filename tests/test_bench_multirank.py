"""bench.py's multi-GPU control flow at world_size 2, on CPU (gloo).

The driver runs `torch.distributed.run --nproc-per-node N bench.py` on an
8-GPU node; no session here has one.  This runs bench.main() itself in two
gloo ranks with the device pieces stood in: the engine by a CPU stand-in that
answers from the oracle (so the parity sample is meaningful and the step
counts are the sequential TimedT's), torch.cuda's synchronisation by no-ops,
the library's RCCL job by nothing (the stand-in all-reduces its statistics
over gloo, as tw_run's reduction does over RCCL).  What is checked is bench.py's
own logic: BASELINE config 3's strong split (one batch over the ranks, rank 0
printing the whole job's line), the weak line measured after it and reported
beside it, the geometry choice per rank share, the barrier + max-over-ranks
timing, and the parity sample rank 0 keeps at N > 1."""
import json
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


class _Stats:
    def __init__(self, **kw):
        self.__dict__.update(kw)


def _worker(rank, world, port, out_path, argv):
    sys.path[:0] = [ROOT, os.path.join(ROOT, "time-warp_amd"), os.path.join(ROOT, "oracle")]
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), WORLD_SIZE=str(world), RANK=str(rank),
                      LOCAL_RANK=str(rank))
    import io
    from contextlib import redirect_stdout

    import torch
    import torch.distributed as dist

    import oracle
    from timewarp import dist as twd
    from timewarp import engine as eng_mod

    real_init, real_reduce = dist.init_process_group, twd.reduce_stats
    dist.init_process_group = lambda backend=None, **kw: real_init("gloo", **kw)
    torch.cuda.set_device = lambda *a, **k: None
    torch.cuda.synchronize = lambda *a, **k: None
    twd.library_comm = lambda world, rank: None
    twd.reduce_stats = lambda local, device=None: real_reduce(local)

    class FakeEngine:
        """tw_run's contract on CPU: the oracle's results, job-wide statistics."""

        def __init__(self, device, comm=None):
            self.geo, self.tie = None, "fifo"

        def load(self, scn, geometry=None):
            self.scn, self.geo = scn, geometry or "dense"
            return self

        def geometry(self):
            return self.geo

        def set_tie_mode(self, t):
            self.tie = t
            return self

        def reset(self):
            pass

        def run(self):
            self.res, self.h = oracle.run_batch(self.scn, threads=2)
            r = self.res
            loc = {"events": int(r["events"].sum()), "delivered": int(r["delivered"].sum()),
                   "dropped": int(r["dropped"].sum()), "undeliverable": int(r["undeliverable"].sum()),
                   "replicas_error": int((r["status"] >= 3).sum())}
            job = real_reduce(loc)
            return _Stats(events=int(job["events"]), delivered=int(job["delivered"]), dropped=int(job["dropped"]),
                          undeliverable=int(job["undeliverable"]),
                          sends=int(job["delivered"] + job["dropped"] + job["undeliverable"]), launches=1,
                          replicas_error=int(job["replicas_error"]))

        def results(self):
            return self.res

        def hashes(self):
            return self.h

        def launch_ms(self):
            return np.array([1.0])

        def lpb_windows(self):
            return (1, 1)

        def close(self):
            pass

    eng_mod.Engine = FakeEngine
    import bench

    sys.argv = ["bench.py"] + argv
    buf = io.StringIO()
    with redirect_stdout(buf):
        bench.main()
    if rank == 0:
        with open(out_path, "w") as f:
            f.write(buf.getvalue())


@pytest.mark.parametrize("weak", [False, True])
def test_bench_two_ranks(tmp_path, oracle_mod, weak):
    out = str(tmp_path / "line.txt")
    argv = ["--config", "token_ring", "--replicas", "8", "--nodes", "8", "--duration-s", "5", "--host-tables",
            "--steps", "1", "--warmup", "0", "--cpu-seconds", "1"] + (["--weak"] if weak else [])
    mp.spawn(_worker, args=(2, _free_port(), out, argv), nprocs=2, join=True)
    lines = [ln for ln in open(out).read().splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    from timewarp import scenarios

    assert d["n_gpus"] == 2 and d["steps"] == 1
    # the whole job's events: one batch of 8 replicas (strong) or 8 per rank (weak)
    total = 16 if weak else 8
    scn = scenarios.token_ring(n_nodes=8, n_replicas=total, launch_duration=5_000_000, drop_log2=10)
    ores, _ = oracle_mod.run_batch(scn, threads=4)
    assert d["config"]["events_per_step"] == int(ores["events"].sum())
    assert d["config"]["replicas_total"] == total
    assert d["config"]["replicas_rank0"] == (8 if weak else 4)
    assert d["scaling"] == ("weak" if weak else "strong")
    # batched logical processes for a share of <= 8,192 replicas (a power of two)
    assert d["config"]["geometry"] == "lpb"
    assert d["parity_sample"]["bit_exact"] and "rank 0" in d["parity_sample"]["against"]
    assert "cpu_baseline" not in d  # rank 0 at N = 1 only
    if weak:
        assert "weak_line" not in d
    else:
        assert d["config"]["baseline_config"] is None  # (only the 65,536-replica batch is config 3)
        w = d["weak_line"]
        assert w["scaling"] == "weak" and w["replicas_per_gpu"] == 8 and w["replicas_total"] == 16
        assert w["value"] > 0 and w["ms_per_step"] > 0
