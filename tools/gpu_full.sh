export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu -x --timeout 200 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?; echo "pytest=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1; rc=$?; echo "smoke=$rc"
if [ $rc -ne 0 ]; then exit $rc; fi
timeout -k 10 400 python bench.py --config hotspot > gpurun_out/bench_c5.log 2>&1; rc=$?; echo "c5=$rc"
exit $rc
