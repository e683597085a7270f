export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5b -o run -- python3 bench.py --config hotspot --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_c5b.log 2>&1; rc=$?; echo "prof=$rc"
[ $rc -eq 0 ] || exit $rc
TW_LIB=$PWD/time-warp_amd/lib/libtimewarp_stats.so timeout -k 10 400 python -u tools/stats_probe.py lpb_hotspot 4096 256 > gpurun_out/stats_c5_lpb2.log 2>&1; rc=$?; echo "stats=$rc"
exit $rc
