"""Summarise a rocprofv3 kernel trace (``--kernel-trace --output-format csv``).

Per kernel name: launches, total/avg time.  For the event kernel (the name
containing ``tw_run_kernel``): the launch-duration histogram and the longest
launches with their position in the launch sequence, so a window loop's time
can be split into its few heavy windows and its many light ones.  Also the
device idle time between consecutive kernels (dispatch gaps).

usage: python tools/trace_summary.py <run_kernel_trace.csv> [--last-frac F]
  --last-frac F: only the last fraction F of the trace's time span (e.g. the
  final bench step)
"""
import csv
import sys
from collections import defaultdict


def short(name: str) -> str:
    n = name.replace("void ", "").replace("(anonymous namespace)::", "")
    return n.split("(")[0][:60]


def main():
    path = sys.argv[1]
    last = None
    if "--last-frac" in sys.argv:
        last = float(sys.argv[sys.argv.index("--last-frac") + 1])
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    if last is not None and rows:
        t0, t1 = rows[0][0], max(e for _, e, _ in rows)
        cut = t1 - (t1 - t0) * last
        rows = [r for r in rows if r[0] >= cut]
    per = defaultdict(lambda: [0, 0])
    ev = []
    gap = 0
    prev_end = None
    for s, e, n in rows:
        k = short(n)
        per[k][0] += 1
        per[k][1] += e - s
        if "tw_run_kernel" in n:
            ev.append((e - s, len(ev)))
        if prev_end is not None and s > prev_end:
            gap += s - prev_end
        prev_end = e if prev_end is None else max(prev_end, e)
    span = (rows[-1][1] - rows[0][0]) if rows else 0
    print(f"span {span / 1e6:.3f} ms, kernels {len(rows)}, idle gaps {gap / 1e6:.3f} ms")
    for k, (c, t) in sorted(per.items(), key=lambda x: -x[1][1]):
        print(f"  {k:40s} {c:7d} launches {t / 1e6:10.3f} ms  avg {t / max(c, 1) / 1e3:9.2f} us")
    if ev:
        tot = sum(d for d, _ in ev)
        buckets = [(0, 20e3), (20e3, 50e3), (50e3, 100e3), (100e3, 300e3), (300e3, 1e6), (1e6, 3e6), (3e6, 1e12)]
        print("event-kernel launch durations:")
        for lo, hi in buckets:
            sel = [d for d, _ in ev if lo <= d < hi]
            print(f"  [{lo / 1e3:7.0f}, {hi / 1e3:9.0f}) us: {len(sel):6d} launches {sum(sel) / 1e6:9.3f} ms "
                  f"({100 * sum(sel) / max(tot, 1):5.1f} %)")
        top = sorted(ev, reverse=True)[:24]
        print("longest event launches (us @ launch index):",
              " ".join(f"{d / 1e3:.0f}@{i}" for d, i in sorted(top, key=lambda x: x[1])))


if __name__ == "__main__":
    main()
