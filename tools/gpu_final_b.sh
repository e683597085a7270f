# round-2 measurement pass B: C5 / C4 traffic passes and bench lines, C2 line
export TMPDIR=/tmp
O=gpurun_out/r02f
mkdir -p $O profiles/r02f/c5 profiles/r02f/c4 profiles/r02f/c2
bash tools/pmc_traffic.sh $O/pmc_c5 --config hotspot > $O/pmc_c5.log 2>&1; rc=$?; echo "pmc_c5=$rc"
[ $rc -eq 0 ] || exit $rc
cp $O/pmc_c5/summary.json profiles/r02f/c5/pmc_summary.json
bash tools/pmc_traffic.sh $O/pmc_c4 --config gossip > $O/pmc_c4.log 2>&1; rc=$?; echo "pmc_c4=$rc"
[ $rc -eq 0 ] || exit $rc
cp $O/pmc_c4/summary.json profiles/r02f/c4/pmc_summary.json
bash tools/pmc_traffic.sh $O/pmc_c2 --config ping_pong > $O/pmc_c2.log 2>&1; rc=$?; echo "pmc_c2=$rc"
[ $rc -eq 0 ] || exit $rc
cp $O/pmc_c2/summary.json profiles/r02f/c2/pmc_summary.json
timeout -k 10 500 python bench.py --config hotspot > $O/bench_c5.log 2>&1; rc=$?; echo "bench_c5=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --config gossip > $O/bench_c4.log 2>&1; rc=$?; echo "bench_c4=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 500 python bench.py --config ping_pong > $O/bench_c2.log 2>&1; rc=$?; echo "bench_c2=$rc"
exit $rc
