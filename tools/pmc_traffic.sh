#!/bin/bash
# HBM traffic of a bench workload: the kernel-stats pass and the FETCH_SIZE /
# WRITE_SIZE passes (separate --pmc runs, kernel trace only), summarised by
# tools/pmc_summary.py with the workload key and engine digest bench.py checks.
# usage: tools/pmc_traffic.sh OUTDIR [bench args...]
set -e
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --no-cpu-baseline $*"
i=2
for P in FETCH_SIZE WRITE_SIZE; do
  i=$((i+1))
  timeout -s KILL 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/pass$i -o run -- python3 bench.py $ARGS > $OUT/pass$i.log 2>&1
  echo "pass $i rc=$?"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 bench.py $ARGS > $OUT/stats.log 2>&1
echo "stats rc=$?"
python3 tools/pmc_summary.py $OUT/summary.json $OUT/stats $OUT/pass3 $OUT/pass4 > $OUT/summary.log 2>&1
python3 bench.py --workload-key $* > $OUT/workload.json
python3 - "$OUT/summary.json" "$*" "$OUT/workload.json" <<'PY'
import json, sys
s = json.load(open(sys.argv[1])); s["bench_args"] = sys.argv[2]; s["steps"] = 1
s.update(json.load(open(sys.argv[3])))
json.dump(s, open(sys.argv[1], "w"), indent=1)
PY
