# round-3 GPU session C: wave K=4 diagnosis (rest), pqueue mode, compact geometry, C2 A/B
export TMPDIR=/tmp
O=gpurun_out/r03c
mkdir -p $O
for a in "16 4 40" "40 4 60" "64 2 30"; do
  TW_WAVE_K=4 timeout -k 10 120 python -u tools/debug_wave_k.py $a >> $O/debug_k4.log 2>&1; rc=$?; echo "debug_k4 $a=$rc"
  [ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
done
timeout -k 10 400 python -u -m pytest tests/test_gpu_pqueue.py -x -v --timeout 300 --timeout-method thread > $O/pqueue.log 2>&1; rc=$?; echo "pqueue=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread -k compact > $O/compact.log 2>&1; rc=$?; echo "compact=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 300 python bench.py --config ping_pong --steps 2 --warmup 1 --no-cpu-baseline > $O/c2_compact.log 2>&1; rc=$?; echo "c2_compact=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --config ping_pong --steps 2 --warmup 1 --no-cpu-baseline --geometry dense > $O/c2_dense.log 2>&1; rc=$?; echo "c2_dense=$rc"
exit $rc
