# round-3 GPU session M: LP binding cache + LDS handler table + one-deep link tables without ordinals;
# the LP event kernel at one wave per SIMD (no scratch) as an A/B library
export TMPDIR=/tmp
O=gpurun_out/r03m
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lpb.py tests/test_gpu_gossip.py -x -q --timeout 300 --timeout-method thread > $O/tests_lp.log 2>&1; rc=$?; echo "tests_lp=$rc"
[ $rc -eq 0 ] || exit $rc
for v in "" lp1; do
  if [ -n "$v" ]; then export TW_LIB=time-warp_amd/lib/libtimewarp_$v.so; fi
  timeout -k 10 300 python3 -u bench.py --config hotspot --steps 2 --warmup 1 --no-cpu-baseline > $O/c5$v.log 2>&1; rc=$?; echo "c5$v=$rc"
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python3 -u bench.py --config gossip --steps 3 --warmup 1 --no-cpu-baseline > $O/c4$v.log 2>&1; rc=$?; echo "c4$v=$rc"
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python3 -u bench.py --replicas 8192 --geometry lpb --steps 2 --warmup 1 --no-cpu-baseline > $O/lpb8k$v.log 2>&1; rc=$?; echo "lpb8k$v=$rc"
  [ $rc -eq 0 ] || exit $rc
done
unset TW_LIB
timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/c3.log 2>&1; rc=$?; echo "c3=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/gpu_all.log 2>&1; rc=$?; echo "gpu_all=$rc"
exit $rc
