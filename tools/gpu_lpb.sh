export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_lpb.py -x -v --timeout 120 --timeout-method thread > gpurun_out/lpb_tests.log 2>&1; rc=$?; echo "lpb_tests=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 600 python -u -m pytest tests/test_gpu_gossip.py -x -q --timeout 120 --timeout-method thread > gpurun_out/gossip_tests.log 2>&1; rc=$?; echo "gossip=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config hotspot --geometry lpb --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/benchq_c5_lpb.log 2>&1; rc=$?; echo "c5lpb=$rc"
exit $rc
