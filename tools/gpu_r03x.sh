# round-3 GPU session X: LP records contiguous per lane (after W: LP scalar blocks)
export TMPDIR=/tmp
O=gpurun_out/r03x
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_lpb.py tests/test_gpu_gossip.py tests/test_gpu_multi.py tests/test_gpu_fullshape.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --config gossip --steps 3 --warmup 1 --no-cpu-baseline > $O/c4.log 2>&1; rc=$?; echo "c4=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --config hotspot --steps 2 --warmup 1 --no-cpu-baseline > $O/c5.log 2>&1; rc=$?; echo "c5=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --replicas 8192 --steps 2 --warmup 1 --no-cpu-baseline > $O/lpb8k.log 2>&1; rc=$?; echo "lpb8k=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 bash tools/pmc_traffic.sh $O/c4_traffic --config gossip > $O/c4_traffic.log 2>&1; rc=$?; echo "c4_traffic=$rc"
cat $O/c4_traffic/summary.log | tail -5
exit $rc
