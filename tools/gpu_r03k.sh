# round-3 GPU session K: device-loop ticks as hipGraphs (A/B against host launches)
export TMPDIR=/tmp
O=gpurun_out/r03k
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_lpb.py tests/test_gpu_gossip.py tests/test_gpu_multi.py -x -q --timeout 300 --timeout-method thread > $O/tests.log 2>&1; rc=$?; echo "tests=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --replicas 8192 --geometry lpb --steps 2 --warmup 1 --no-cpu-baseline > $O/lpb8k.log 2>&1; rc=$?; echo "lpb8k=$rc"
[ $rc -eq 0 ] || exit $rc
TW_NO_GRAPH=1 timeout -k 10 300 python3 -u bench.py --replicas 8192 --geometry lpb --steps 2 --warmup 1 --no-cpu-baseline > $O/lpb8k_nograph.log 2>&1; rc=$?; echo "lpb8k_ng=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/lpb8k -o run -- python3 bench.py --replicas 8192 --geometry lpb --steps 1 --warmup 1 --no-cpu-baseline > $O/lpb8k_prof.log 2>&1; rc=$?; echo "lpb8k_prof=$rc"
[ $rc -eq 0 ] || exit $rc
python3 tools/trace_summary.py $O/lpb8k/run_kernel_trace.csv --last-frac 0.45 > $O/lpb8k_trace.txt 2>&1
timeout -k 10 300 python3 -u bench.py --config gossip --steps 3 --warmup 1 --no-cpu-baseline > $O/c4.log 2>&1; rc=$?; echo "c4=$rc"
[ $rc -eq 0 ] || exit $rc
TW_NO_GRAPH=1 timeout -k 10 300 python3 -u bench.py --config gossip --steps 3 --warmup 1 --no-cpu-baseline > $O/c4_nograph.log 2>&1; rc=$?; echo "c4_ng=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --config hotspot --steps 2 --warmup 1 --no-cpu-baseline > $O/c5.log 2>&1; rc=$?; echo "c5=$rc"
exit $rc
