# round-3 GPU session Z: instruction counts of an interpreter pass (PMC, pass probe k=0 vs k=16 extra traces)
export TMPDIR=/tmp
O=gpurun_out/r03z
mkdir -p $O
export PROBE_REPS=1
for k in 0 16; do
  PROBE_KS=$k timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_WAVE_CYCLES SQ_WAVES --kernel-trace --output-format csv -d $O/k$k -o run -- python3 tools/pass_probe.py 64 1024 100 lpb trace > $O/k$k.log 2>&1; rc=$?; echo "k$k=$rc"
  [ $rc -eq 0 ] || exit $rc
done
for k in 0 16; do
  PROBE_KS=$k timeout -s KILL 120 rocprofv3 --pmc SQ_WAIT_INST_ANY SQ_BUSY_CYCLES SQ_INST_CYCLES_SALU SQ_WAIT_ANY --kernel-trace --output-format csv -d $O/w$k -o run -- python3 tools/pass_probe.py 64 1024 100 lpb trace > $O/w$k.log 2>&1; rc=$?; echo "w$k=$rc"
  [ $rc -eq 0 ] || exit $rc
done
exit 0
