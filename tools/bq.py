"""Summarise bench.py JSON lines from logs: value (G events/s), ms per step,
parity sample.  usage: python tools/bq.py gpurun_out/benchq_c5*.log"""
import json
import sys

for f in sys.argv[1:]:
    try:
        line = next(l for l in open(f) if l.startswith("{"))
    except (OSError, StopIteration):
        print(f"{f}: no bench line")
        continue
    d = json.loads(line)
    ps = d.get("parity_sample")
    print(f"{f}: {d['value'] / 1e9:.3f} G  {d['ms_per_step']:.2f} ms"
          + (f"  parity {ps}" if ps else ""))
