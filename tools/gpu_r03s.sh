# round-3 GPU session S: LP lanes with the opcode-uniform interpreter pass (A/B library), pass-cost probe on both
export TMPDIR=/tmp
O=gpurun_out/r03s
mkdir -p $O
for v in "" nopl; do
  if [ -n "$v" ]; then export TW_LIB=time-warp_amd/lib/libtimewarp_$v.so; fi
  timeout -k 10 300 python3 -u bench.py --config hotspot --steps 1 --warmup 1 --no-cpu-baseline > $O/c5$v.log 2>&1; rc=$?; echo "c5$v=$rc"
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python3 -u bench.py --config gossip --steps 3 --warmup 1 --no-cpu-baseline > $O/c4$v.log 2>&1; rc=$?; echo "c4$v=$rc"
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python3 -u bench.py --replicas 8192 --steps 2 --warmup 1 --no-cpu-baseline > $O/lpb8k$v.log 2>&1; rc=$?; echo "lpb8k$v=$rc"
  [ $rc -eq 0 ] || exit $rc
  timeout -k 10 300 python3 -u tools/pass_probe.py 64 4096 200 > $O/pass_probe$v.log 2>&1; rc=$?; echo "probe$v=$rc"
  [ $rc -eq 0 ] || exit $rc
done
unset TW_LIB
TW_LIB=time-warp_amd/lib/libtimewarp_nopl.so timeout -k 10 300 python -u -m pytest tests/test_gpu_lpb.py tests/test_gpu_gossip.py -x -q --timeout 300 --timeout-method thread > $O/tests_nopl.log 2>&1; rc=$?; echo "tests_nopl=$rc"
exit $rc
