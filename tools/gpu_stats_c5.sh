export TMPDIR=/tmp
mkdir -p gpurun_out
TW_LIB=$PWD/time-warp_amd/lib/libtimewarp_stats.so timeout -k 10 400 python -u tools/stats_probe.py lpb_hotspot 4096 256 > gpurun_out/stats_c5_lpb.log 2>&1; rc=$?; echo "stats=$rc"
exit $rc
