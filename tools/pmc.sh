#!/bin/bash
# PMC passes for the bench workload (separate --pmc runs; kernel-trace only, no sys/runtime trace).
# usage: tools/pmc.sh OUTDIR [bench args...]
set -e
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
ARGS="--steps 1 --warmup 0 --no-cpu-baseline $*"
i=0
for P in "SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_INSTS_SMEM GRBM_GUI_ACTIVE" \
         "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_LDS_BANK_CONFLICT SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES" \
         "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/pass$i -o run -- python3 bench.py $ARGS > $OUT/pass$i.log 2>&1
  echo "pass $i rc=$?"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/stats -o run -- python3 bench.py $ARGS > $OUT/stats.log 2>&1
echo "stats rc=$?"
python3 tools/pmc_summary.py $OUT/summary.json $OUT/stats $OUT/pass1 $OUT/pass2 $OUT/pass3 $OUT/pass4 $OUT/pass5 > $OUT/summary.log 2>&1
# provenance: the engine build and workload these counters belong to (bench.py
# uses the summary for roofline.traffic only when both match)
python3 bench.py --workload-key $* > $OUT/workload.json
python3 - "$OUT/summary.json" "$*" "$OUT/workload.json" <<'PY'
import json, sys
s = json.load(open(sys.argv[1])); s["bench_args"] = sys.argv[2]; s["steps"] = 1
s.update(json.load(open(sys.argv[3])))
json.dump(s, open(sys.argv[1], "w"), indent=1)
PY
