export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3lpb -o run -- python3 bench.py --replicas 8192 --geometry lpb --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_c3lpb.log 2>&1; rc=$?; echo "prof=$rc"
exit $rc
