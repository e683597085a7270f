# round-3 GPU session T: no load left in flight into the step (far_pop drained, throw_to drained):
# the interpreter passes no longer wait vmcnt(0) at their top (tools/waitcnt_audit.py)
export TMPDIR=/tmp
O=gpurun_out/r03t
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_lpb.py tests/test_gpu_gossip.py tests/test_gpu_parity.py tests/test_gpu_programs.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/pass_probe.py 64 4096 200 > $O/pass_probe.log 2>&1; rc=$?; echo "probe=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --config hotspot --steps 2 --warmup 1 --no-cpu-baseline > $O/c5.log 2>&1; rc=$?; echo "c5=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --config gossip --steps 3 --warmup 1 --no-cpu-baseline > $O/c4.log 2>&1; rc=$?; echo "c4=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --replicas 8192 --steps 2 --warmup 1 --no-cpu-baseline > $O/lpb8k.log 2>&1; rc=$?; echo "lpb8k=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --steps 3 --warmup 1 --no-cpu-baseline > $O/c3.log 2>&1; rc=$?; echo "c3=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --config ping_pong --steps 3 --warmup 1 --no-cpu-baseline > $O/c2.log 2>&1; rc=$?; echo "c2=$rc"
exit $rc
