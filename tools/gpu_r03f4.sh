# round-3 final pass 4 (engine with the SEND, ALU/NSTORE and TRACE pairs fused + device-drawn tables).
# usage: bash tools/gpu_r03f3.sh PART   (A: tests + smoke + quick C3 line; B: C3 PMC + C2 traffic;
#        C: C4/C5 traffic + C3 kernel stats; D: bench lines + multi-device tests + C3-8k trace)
export TMPDIR=/tmp
O=gpurun_out/r03f4
mkdir -p $O
run() {  # run NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name=$rc"
  [ $rc -eq 0 ] || exit $rc
}
case $1 in
A)
  run pytest_gpu 900 python -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  run bq_c3 300 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
  ;;
S)
  run smoke 300 python -c "import __graft_entry__ as g; g.smoke()"
  ;&
B)
  bash tools/pmc.sh $O/pmc > $O/pmc.log 2>&1; rc=$?; echo "pmc=$rc"; [ $rc -eq 0 ] || exit $rc
  bash tools/pmc_traffic.sh $O/pmct_c2 --config ping_pong > $O/pmct_c2.log 2>&1; rc=$?; echo "pmct_c2=$rc"; [ $rc -eq 0 ] || exit $rc
  ;&
C)
  bash tools/pmc_traffic.sh $O/pmct_c4 --config gossip > $O/pmct_c4.log 2>&1; rc=$?; echo "pmct_c4=$rc"; [ $rc -eq 0 ] || exit $rc
  bash tools/pmc_traffic.sh $O/pmct_c5 --config hotspot > $O/pmct_c5.log 2>&1; rc=$?; echo "pmct_c5=$rc"; [ $rc -eq 0 ] || exit $rc
  ;;
D)
  run bench_c3 500 python3 -u bench.py
  run bench_c2 300 python3 -u bench.py --config ping_pong
  run bench_c4 300 python3 -u bench.py --config gossip
  run bench_c5 400 python3 -u bench.py --config hotspot --steps 2 --warmup 1
  run bench_c3_8k 300 python3 -u bench.py --replicas 8192
  run tests_multi 300 python -u -m pytest tests/test_gpu_multi.py -x -q --timeout 300 --timeout-method thread
  ;;
esac
exit 0
