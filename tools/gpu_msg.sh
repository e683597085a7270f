export TMPDIR=/tmp
O=gpurun_out/r02f
mkdir -p $O profiles/r02f/c3_msg
bash tools/pmc_traffic.sh $O/pmc_c3msg --duration-s 24576 --drop-log2 16 > $O/pmc_c3msg.log 2>&1; rc=$?; echo "pmc=$rc"
[ $rc -eq 0 ] || exit $rc
cp $O/pmc_c3msg/summary.json profiles/r02f/c3_msg/pmc_summary.json
timeout -k 10 600 python bench.py --duration-s 24576 --drop-log2 16 --steps 2 --warmup 1 > $O/bench_c3_msg.log 2>&1; rc=$?; echo "bench=$rc"
exit $rc
