"""Diagnostic: the wave kernel at a given near-queue depth (TW_WAVE_K) against
the oracle on hotspot batches whose receiver backlog exceeds the on-chip
queue; prints every replica and field that differs.
usage: TW_WAVE_K=4 python tools/debug_wave_k.py [senders] [replicas] [msgs]"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "time-warp_amd"), os.path.join(ROOT, "oracle")]

import numpy as np  # noqa: E402

import oracle  # noqa: E402  (checker)
from timewarp import scenarios  # noqa: E402
from timewarp.abi import RESULT_FIELDS  # noqa: E402
from timewarp.engine import Engine  # noqa: E402


def main():
    S = int(sys.argv[1]) if len(sys.argv) > 1 else 64
    R = int(sys.argv[2]) if len(sys.argv) > 2 else 8
    M = int(sys.argv[3]) if len(sys.argv) > 3 else 60
    scn = scenarios.hotspot(n_senders=S, n_replicas=R, msg_num=M)
    ores, oh = oracle.run_batch(scn, threads=8)
    for geo in ("wave", "dense"):
        with Engine(0) as e:
            e.load(scn, geometry=geo)
            e.run()
            res, h = e.results(), e.hashes()
        bad = 0
        for f in RESULT_FIELDS:
            if f == "tie_flags":
                continue
            m = np.nonzero(res[f] != ores[f])[0]
            if m.size:
                bad += 1
                print(geo, f, "replicas", m[:8].tolist(), "gpu", res[f][m[:8]].tolist(), "oracle",
                      ores[f][m[:8]].tolist(), flush=True)
        hm = np.nonzero((h != oh).any(axis=1))[0]
        print(geo, "K", os.environ.get("TW_WAVE_K"), "S", S, "R", R, "M", M, "bad fields", bad, "hash replicas",
              hm[:8].tolist(), "status", np.unique(res["status"]).tolist(), flush=True)


if __name__ == "__main__":
    main()
