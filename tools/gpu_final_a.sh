# round-2 measurement pass A: tests, smoke, C3 PMC passes, C3 bench line
export TMPDIR=/tmp
O=gpurun_out/r02f
mkdir -p $O profiles/r02f
timeout -k 10 900 python -u -m pytest tests/ -q -m gpu -x --timeout 200 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; echo "pytest=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1; rc=$?; echo "smoke=$rc"
[ $rc -eq 0 ] || exit $rc
bash tools/pmc.sh $O/pmc_c3 > $O/pmc_c3.log 2>&1; rc=$?; echo "pmc_c3=$rc"
[ $rc -eq 0 ] || exit $rc
cp $O/pmc_c3/summary.json profiles/r02f/pmc_summary.json
timeout -k 10 500 python bench.py > $O/bench_c3.log 2>&1; rc=$?; echo "bench_c3=$rc"
exit $rc
