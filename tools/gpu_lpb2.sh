export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_lpb.py tests/test_gpu_gossip.py -x -q --timeout 200 --timeout-method thread > gpurun_out/lpb_tests.log 2>&1; rc=$?; echo "lpb_tests=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --replicas 8192 --geometry lpb --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/benchq_c3_8k_lpb.log 2>&1; rc=$?; echo "c3_8k_lpb=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config gossip --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/benchq_c4.log 2>&1; rc=$?; echo "c4=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python bench.py --config hotspot --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/benchq_c5.log 2>&1; rc=$?; echo "c5=$rc"
exit $rc
