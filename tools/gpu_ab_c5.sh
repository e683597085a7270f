export TMPDIR=/tmp
mkdir -p gpurun_out
TW_LIB=$PWD/time-warp_amd/lib/libtimewarp_old.so timeout -k 10 300 python bench.py --config hotspot --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab_c5_old.log 2>&1; rc=$?; echo "old=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config hotspot --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/ab_c5_new.log 2>&1; rc=$?; echo "new=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -u -m pytest tests/test_gpu_lpb.py tests/test_gpu_gossip.py -x -q --timeout 200 --timeout-method thread > gpurun_out/lpb_tests.log 2>&1; rc=$?; echo "lpb_tests=$rc"
exit $rc
