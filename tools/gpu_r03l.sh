# round-3 GPU session L: LP event-path cycle splits (SEND / DELIVER / due pop / lane prologue and epilogue)
export TMPDIR=/tmp
O=gpurun_out/r03l
mkdir -p $O
export TW_LIB=time-warp_amd/lib/libtimewarp_stats.so
timeout -k 10 300 python3 -u tools/stats_probe.py lpb_hotspot 4096 > $O/stats_lpb_hotspot.log 2>&1; rc=$?; echo "c5=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/stats_probe.py gossip > $O/stats_gossip.log 2>&1; rc=$?; echo "c4=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/stats_probe.py lpb_token 8192 > $O/stats_lpb_token.log 2>&1; rc=$?; echo "c3=$rc"
exit $rc
