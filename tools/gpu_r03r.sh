# round-3 GPU session R: per-pass cost on the hotspot receiver's chain
export TMPDIR=/tmp
O=gpurun_out/r03r
mkdir -p $O
timeout -k 10 400 python3 -u tools/pass_probe.py 64 4096 200 > $O/pass_probe.log 2>&1; rc=$?; echo "probe=$rc"
exit $rc
