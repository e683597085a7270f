# round-3 GPU session C: wave-kernel regression bisect (current vs round-2 wave.hip), LP due-sort validation
export TMPDIR=/tmp
O=gpurun_out/r03c
mkdir -p $O
for L in oldwave default; do
  if [ $L = default ]; then unset TW_LIB; else export TW_LIB=$PWD/time-warp_amd/lib/libtimewarp_$L.so; fi
  timeout -k 10 300 python -u -m pytest tests/test_gpu_gossip.py -x -q --timeout 120 --timeout-method thread -k "replica_engine" > $O/gossip_$L.log 2>&1; rc=$?; echo "gossip_$L=$rc"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  TW_WAVE_K=4 timeout -k 10 120 python -u tools/debug_wave_k.py 64 8 60 > $O/debug_k4_$L.log 2>&1; rc=$?; echo "debugk4_$L=$rc"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
  TW_WAVE_K=32 TW_GEOMETRY=wave timeout -k 10 120 python -u tools/debug_wave_k.py 256 4 200 > $O/debug_k32_$L.log 2>&1; rc=$?; echo "debugk32_$L=$rc"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
unset TW_LIB
timeout -k 10 600 python -u -m pytest tests/test_gpu_lpb.py tests/test_gpu_fullshape.py -x -q --timeout 300 --timeout-method thread -k "lpb" > $O/lpb_tests.log 2>&1; rc=$?; echo "lpb_tests=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --config hotspot --steps 2 --warmup 1 --no-cpu-baseline > $O/c5.log 2>&1; rc=$?; echo "c5=$rc"
exit $rc
