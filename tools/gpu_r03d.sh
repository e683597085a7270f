# round-3 GPU session D: wave kernel after the SCC-clobber fix, then the whole GPU suite + smoke
export TMPDIR=/tmp
O=gpurun_out/r03d
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_gossip.py -x -q --timeout 120 --timeout-method thread -k "replica_engine" > $O/gossip.log 2>&1; rc=$?; echo "gossip=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
TW_WAVE_K=4 timeout -k 10 120 python -u tools/debug_wave_k.py 64 8 60 > $O/debug_k4.log 2>&1; rc=$?; echo "debugk4=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_gpu_wave_k.py tests/test_gpu_pqueue.py -x -q --timeout 200 --timeout-method thread > $O/wavek.log 2>&1; rc=$?; echo "wavek=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -q --timeout 300 --timeout-method thread > $O/gpu_all.log 2>&1; rc=$?; echo "gpu_all=$rc"
[ $rc -eq 0 ] || [ $rc -eq 1 ] || exit $rc
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1; rc=$?; echo "smoke=$rc"
exit $rc
