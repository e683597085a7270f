# round-3 GPU session AB: tw_run's statistics reduced on the device (no per-replica results copy in the timed step)
export TMPDIR=/tmp
O=gpurun_out/r03ab
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_programs.py tests/test_gpu_multi.py tests/test_gpu_gossip.py tests/test_gpu_abi2.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --config ping_pong --steps 3 --warmup 1 --no-cpu-baseline > $O/c2.log 2>&1; rc=$?; echo "c2=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/c3.log 2>&1; rc=$?; echo "c3=$rc"
exit $rc
