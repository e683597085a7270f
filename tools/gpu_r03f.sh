# round-3 GPU session F: where C3's batched-LP loop spends its time at 8,192 replicas (per-kernel stats)
export TMPDIR=/tmp
O=gpurun_out/r03f
mkdir -p $O
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $O/lpb8k -o run -- python3 bench.py --replicas 8192 --geometry lpb --steps 1 --warmup 0 --no-cpu-baseline > $O/lpb8k.log 2>&1; rc=$?; echo "lpb8k=$rc"
exit $rc
