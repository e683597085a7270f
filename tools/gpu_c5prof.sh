export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 bench.py --config hotspot --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_c5.log 2>&1; rc=$?; echo "prof_c5=$rc"
exit $rc
