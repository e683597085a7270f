#!/usr/bin/env python3
"""Turn the PMC passes over tools/ubench/pmc_calib into a calibration table.

usage: pmc_calib.py OUT.json RUN_LOG FETCH_DIR WRITE_DIR

RUN_LOG holds the ubench's "<kernel> bytes_read=.. bytes_written=.." lines;
FETCH_DIR / WRITE_DIR are the rocprofv3 output directories of the FETCH_SIZE
and WRITE_SIZE passes.  For each kernel: the algorithmic bytes, the counter in
bytes (KiB x 1024) and their ratio -- the factor tools/pmc_summary.py applies.
"""
import csv
import glob
import json
import os
import re
import sys


def counter(d, name):
    """{kernel: counter value per dispatch} (write_stream also runs once as the
    buffer's first touch: every dispatch moves the same bytes, so average)"""
    vals, n = {}, {}
    for f in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        for row in csv.DictReader(open(f)):
            if row.get("Counter_Name") != name:
                continue
            k = row.get("Kernel_Name", "").split("(")[0].split(" ")[-1]
            vals[k] = vals.get(k, 0.0) + float(row["Counter_Value"])
            n[k] = n.get(k, 0) + 1
    return {k: v / n[k] for k, v in vals.items()}


def main():
    out, log, fdir, wdir = sys.argv[1:]
    algo = {}
    for line in open(log):
        m = re.match(r"(\w+) bytes_read=(\d+) bytes_written=(\d+)", line)
        if m:
            algo[m.group(1)] = (int(m.group(2)), int(m.group(3)))
    fetch, write = counter(fdir, "FETCH_SIZE"), counter(wdir, "WRITE_SIZE")
    rows = {}
    for k, (rd, wr) in algo.items():
        f = next((v for n, v in fetch.items() if k in n), None)
        w = next((v for n, v in write.items() if k in n), None)
        rows[k] = {"bytes_read": rd, "bytes_written": wr,
                   "fetch_size_bytes": f * 1024 if f is not None else None,
                   "write_size_bytes": w * 1024 if w is not None else None,
                   "read_over_fetch": rd / (f * 1024) if f and rd else None,
                   "written_over_write": wr / (w * 1024) if w and wr else None}
    json.dump({"ubench": "tools/ubench/pmc_calib.hip (2 GiB buffer, 16 B per lane, coalesced)",
               "counters": "FETCH_SIZE and WRITE_SIZE in separate rocprofv3 --pmc passes (KiB per dispatch)",
               "kernels": rows}, open(out, "w"), indent=1)
    print(json.dumps(rows, indent=1))


if __name__ == "__main__":
    main()
