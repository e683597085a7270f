export TMPDIR=/tmp
mkdir -p gpurun_out
for L in old new; do
  if [ $L = old ]; then export TW_LIB=$PWD/time-warp_amd/lib/libtimewarp_old.so; else unset TW_LIB; fi
  timeout -k 10 300 python bench.py --config hotspot --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab_c5_$L.log 2>&1; rc=$?; echo "c5_$L=$rc"
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python bench.py --config gossip --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_c4_$L.log 2>&1; rc=$?; echo "c4_$L=$rc"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_lpb.py tests/test_gpu_gossip.py -x -q --timeout 200 --timeout-method thread > gpurun_out/lpb_tests.log 2>&1; rc=$?; echo "lpb_tests=$rc"
exit $rc
