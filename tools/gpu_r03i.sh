# round-3 GPU session I: chunked per-replica work-list scan, PRW kernel variant
export TMPDIR=/tmp
O=gpurun_out/r03i
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_lpb.py -x -v --timeout 300 --timeout-method thread > $O/lpb_tests.log 2>&1; rc=$?; echo "lpb_tests=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_gossip.py tests/test_gpu_multi.py tests/test_gpu_fullshape.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lpb8k -o run -- python3 bench.py --replicas 8192 --geometry lpb --steps 2 --warmup 1 --no-cpu-baseline > $O/lpb8k.log 2>&1; rc=$?; echo "lpb8k=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config hotspot --steps 2 --warmup 1 --no-cpu-baseline > $O/c5.log 2>&1; rc=$?; echo "c5=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u bench.py --config gossip --steps 3 --warmup 1 --no-cpu-baseline > $O/c4.log 2>&1; rc=$?; echo "c4=$rc"
exit $rc
