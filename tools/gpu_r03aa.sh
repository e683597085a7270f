# round-3 GPU session AA: batched-LP cross-node forks emitted inside the interpreter pass (main's fork loop inline)
export TMPDIR=/tmp
O=gpurun_out/r03aa
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_lpb.py tests/test_gpu_fullshape.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --replicas 8192 --steps 2 --warmup 1 > $O/lpb8k.log 2>&1; rc=$?; echo "lpb8k=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --config hotspot --steps 2 --warmup 1 --no-cpu-baseline > $O/c5.log 2>&1; rc=$?; echo "c5=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --replicas 16384 --geometry lpb --steps 2 --warmup 1 --no-cpu-baseline > $O/lpb16k.log 2>&1; rc=$?; echo "lpb16k=$rc"
exit $rc
