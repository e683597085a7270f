export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -u -m pytest tests/test_gpu_lpb.py -x -v --timeout 200 --timeout-method thread > gpurun_out/lpb_tests.log 2>&1; rc=$?; echo "lpb_tests=$rc"
exit $rc
