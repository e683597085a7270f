# round-3 final pass, part 2: C2 / C4 / C5 / C3-at-8,192 bench lines (with CPU baselines) and traffic passes
export TMPDIR=/tmp
O=gpurun_out/r03final2
mkdir -p $O
run() {  # run NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name=$rc"
  [ $rc -eq 0 ] || exit $rc
}
timeout -k 10 300 python -u -m pytest tests/test_gpu_multi.py -x -q --timeout 300 --timeout-method thread > $O/tests_multi.log 2>&1; echo "tests_multi=$?"
run bench_c2 300 python3 -u bench.py --config ping_pong
run bench_c4 300 python3 -u bench.py --config gossip
run bench_c5 400 python3 -u bench.py --config hotspot --steps 2 --warmup 1
run bench_c3_8k 300 python3 -u bench.py --replicas 8192
run prof_c3_8k 300 rocprofv3 --kernel-trace --stats --output-format csv -d $O/prof_c3_8k -o run -- python3 bench.py --replicas 8192 --steps 1 --warmup 1 --no-cpu-baseline
python3 tools/trace_summary.py $O/prof_c3_8k/run_kernel_trace.csv --last-frac 0.45 > $O/prof_c3_8k_trace.txt 2>&1
rm -f $O/prof_c3_8k/run_kernel_trace.csv
run pmct_c2 600 bash tools/pmc_traffic.sh $O/pmct_c2 --config ping_pong
run pmct_c5 600 bash tools/pmc_traffic.sh $O/pmct_c5 --config hotspot
run pmct_c4 600 bash tools/pmc_traffic.sh $O/pmct_c4 --config gossip
exit 0
