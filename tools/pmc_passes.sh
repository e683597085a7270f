#!/bin/bash
# Two quick PMC passes (instruction mix, wait/issue cycles; PMC_SET=traffic:
# FETCH_SIZE and WRITE_SIZE) over a 1-step bench
# run; prints per-dispatch sums for the event kernels.
# usage: tools/pmc_passes.sh OUTDIR [bench args...]   (env TW_GEOMETRY etc. pass through)
OUT=$1; shift
mkdir -p $OUT
export TMPDIR=/tmp
i=0
if [ "$PMC_SET" = traffic ]; then SETS=("FETCH_SIZE" "WRITE_SIZE"); else SETS=("SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR SQ_WAVE_CYCLES" \
         "SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_BRANCH SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_SCA SQ_BUSY_CYCLES GRBM_GUI_ACTIVE"); fi
for P in "${SETS[@]}"; do
  i=$((i+1))
  timeout -s KILL 240 rocprofv3 --pmc $P --kernel-trace --output-format csv -d $OUT/q$i -o run -- python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline "$@" > $OUT/q$i.log 2>&1
  rc=$?
  echo "pass $i rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
python3 - $OUT <<'PY'
import csv, glob, sys, collections, json
out = sys.argv[1]
agg = collections.defaultdict(float)
for f in glob.glob(out + "/q*/**/*counter_collection.csv", recursive=True):
    for row in csv.DictReader(open(f)):
        k = row.get("Kernel_Name", "")
        if "tw_run_kernel" in k or "tw_wave_kernel" in k:
            agg[row["Counter_Name"]] += float(row["Counter_Value"])
ev = None
for line in open(out + "/q1.log"):
    if line.startswith("{"):
        ev = json.loads(line)["config"]["events_per_step"]
print(json.dumps({"events": ev, **{k: v for k, v in sorted(agg.items())},
                  "per_event": {k: v / ev for k, v in sorted(agg.items())} if ev else None}, indent=1))
PY
