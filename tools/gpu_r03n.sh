# round-3 GPU session N: hotspot receiver-lane cycle splits; PC sampling of the C3 replica kernel
export TMPDIR=/tmp
O=gpurun_out/r03n
mkdir -p $O
TW_LIB=time-warp_amd/lib/libtimewarp_stats.so timeout -k 10 300 python3 -u tools/stats_probe.py lpb_hotspot 4096 > $O/stats_lpb_hotspot.log 2>&1; rc=$?; echo "stats=$rc"
[ $rc -eq 0 ] || exit $rc
rc=0

exit $rc
