# round-3 GPU session J: where the batched-LP C3 time goes (kernel trace, per-path counters), lpb at 16k/32k replicas
export TMPDIR=/tmp
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lpb8k -o run -- python3 bench.py --replicas 8192 --geometry lpb --steps 1 --warmup 1 --no-cpu-baseline > $O/lpb8k.log 2>&1; rc=$?; echo "lpb8k=$rc"
[ $rc -eq 0 ] || exit $rc
python3 tools/trace_summary.py $O/lpb8k/run_kernel_trace.csv --last-frac 0.45 > $O/lpb8k_trace.txt 2>&1
TW_LIB=time-warp_amd/lib/libtimewarp_stats.so timeout -k 10 300 python3 -u tools/stats_probe.py lpb_token 8192 > $O/stats_lpb_token.log 2>&1; rc=$?; echo "stats=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --replicas 16384 --geometry lpb --steps 2 --warmup 1 --no-cpu-baseline > $O/lpb16k.log 2>&1; rc=$?; echo "lpb16k=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u bench.py --replicas 32768 --geometry lpb --steps 2 --warmup 1 --no-cpu-baseline > $O/lpb32k.log 2>&1; rc=$?; echo "lpb32k=$rc"
exit $rc
