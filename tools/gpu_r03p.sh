# round-3 GPU session P: C5 window-loop kernel trace
export TMPDIR=/tmp
O=gpurun_out/r03p
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $O/c5 -o run -- python3 bench.py --config hotspot --steps 1 --warmup 0 --no-cpu-baseline > $O/c5_prof.log 2>&1; rc=$?; echo "c5_prof=$rc"
[ $rc -eq 0 ] || exit $rc
python3 tools/trace_summary.py $O/c5/run_kernel_trace.csv > $O/c5_trace.txt 2>&1
rm -f $O/c5/run_kernel_trace.csv.gz; gzip -f $O/c5/run_kernel_trace.csv
exit 0
