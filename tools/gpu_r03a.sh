# round-3 GPU session A: new parity tests first, then the whole GPU suite + smoke
export TMPDIR=/tmp
O=gpurun_out/r03a
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_multi.py tests/test_gpu_wave_k.py tests/test_gpu_fullshape.py -x -v --timeout 300 --timeout-method thread -k "multi or rccl or shards or wave_k or device_loop or lpb_full" > $O/new_tests.log 2>&1; rc=$?; echo "new_tests=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke=$rc"
exit $rc
