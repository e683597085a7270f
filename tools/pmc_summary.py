#!/usr/bin/env python3
"""Summarise rocprofv3 output for profiles/.

usage: pmc_summary.py OUT.json KERNEL_STATS_DIR [PMC_DIR ...]

* kernel stats: `rocprofv3 --kernel-trace --stats --output-format csv` (*_kernel_stats.csv)
* PMC passes (tools/pmc.sh): `*counter_collection.csv`, one row per dispatch x counter.
HBM traffic per dispatch: bytes = (2 * FETCH_SIZE + WRITE_SIZE) * 1024.  The
factor 2 on FETCH_SIZE: on gfx950 FETCH_SIZE counts 64 B per 128-B read request
of a wide coalesced stream, i.e. half the bytes, while WRITE_SIZE counts written
bytes exactly.  Measured here, not assumed: tools/ubench/pmc_calib.hip streams
2 GiB with 16 B per lane (the engine's record access shape) and
profiles/pmc_calibration.json holds the result: bytes read / (FETCH_SIZE x 1024)
= 2.000, bytes written / (WRITE_SIZE x 1024) = 1.000 (raw counter CSVs in
profiles/r02c/calib/).  FETCH_SIZE and WRITE_SIZE are reported raw beside the
derived value.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def kernel_stats(d):
    out = []
    for f in glob.glob(os.path.join(d, "**", "*kernel_stats.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            out.append({"name": row["Name"], "calls": int(row["Calls"]), "total_ns": float(row["TotalDurationNs"]),
                        "avg_ns": float(row["AverageNs"]), "pct": float(row["Percentage"]),
                        "min_ns": float(row["MinNs"]), "max_ns": float(row["MaxNs"])})
    return sorted(out, key=lambda r: -r["total_ns"])


def counters(d):
    """{counter: {kernel short name: [values per dispatch]}}"""
    res = defaultdict(lambda: defaultdict(list))
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            name = row.get("Kernel_Name", row.get("Kernel-Name", "?"))
            short = "tw_run_kernel" if "tw_run_kernel" in name else name.split("(")[0][-60:]
            cname = row.get("Counter_Name", row.get("Counter-Name"))
            val = float(row.get("Counter_Value", row.get("Counter-Value", 0)))
            res[cname][short].append(val)
    return res


def main():
    out_path, stats_dir, *pmc_dirs = sys.argv[1:]
    summary = {"kernel_stats": kernel_stats(stats_dir), "counters": {}}
    agg = defaultdict(dict)
    for d in pmc_dirs:
        for cname, per_kernel in counters(d).items():
            for k, vals in per_kernel.items():
                agg[k][cname] = {"dispatches": len(vals), "sum": sum(vals), "avg": sum(vals) / max(1, len(vals))}
    summary["counters"] = agg
    run = agg.get("tw_run_kernel", {})
    if "FETCH_SIZE" in run and "WRITE_SIZE" in run:
        fetch, write = run["FETCH_SIZE"]["sum"], run["WRITE_SIZE"]["sum"]
        summary["fetch_size"], summary["write_size"] = fetch, write
        summary["formula"] = "(2*FETCH_SIZE + WRITE_SIZE)*1024"
        summary["hbm_bytes_total"] = (2 * fetch + write) * 1024
        summary["hbm_bytes_per_dispatch"] = summary["hbm_bytes_total"] / max(1, run["FETCH_SIZE"]["dispatches"])
    # window loops (LP / batched LP): every kernel of the loop moves bytes, the
    # event kernel most; their sum is the loop's traffic
    f_all = sum(v["FETCH_SIZE"]["sum"] for k, v in agg.items() if "FETCH_SIZE" in v and "tw_" in k)
    w_all = sum(v["WRITE_SIZE"]["sum"] for k, v in agg.items() if "WRITE_SIZE" in v and "tw_" in k)
    if f_all or w_all:
        summary["hbm_bytes_all_tw"] = (2 * f_all + w_all) * 1024
        summary["fetch_size_all_tw"], summary["write_size_all_tw"] = f_all, w_all
    json.dump(summary, open(out_path, "w"), indent=1)
    print(json.dumps({k: v for k, v in summary.items() if k != "counters"}, indent=1)[:3000])


if __name__ == "__main__":
    main()
