#!/bin/bash
# One rocprofv3 PMC pass per argument over a 1-step bench run (kernel-trace only).
# usage: tools/pmc_quick.sh OUTDIR "CNT1 CNT2 ..." ["CNT ..."]...
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
i=0
for P in "$@"; do
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/q$i -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline > $OUT/q$i.log 2>&1
  rc=$?
  echo "pass $i ($P) rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections
out = sys.argv[1]
agg = collections.defaultdict(float)
for f in glob.glob(out + "/q*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        if "tw_run_kernel" in row.get("Kernel_Name", ""):
            agg[row["Counter_Name"]] += float(row["Counter_Value"])
for k, v in sorted(agg.items()):
    print(f"{k} {v:.6g}")
PY
