set -e
mkdir -p gpurun_out
L=$PWD/time-warp_amd/lib
for v in base new base new; do
  if [ $v = base ]; then export TW_LIB=$L/libtimewarp_base.so; else export TW_LIB=$L/libtimewarp.so; fi
  timeout -k 10 200 python bench.py --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab1_$v.log 2>&1
  grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab1_$v.log >> gpurun_out/ab1_summary.txt
  echo "$v" >> gpurun_out/ab1_summary.txt
done
export TW_PROBE_TIE=forkfirst
TW_LIB=$L/libtimewarp_base_stats.so timeout -k 10 300 python tools/stats_probe.py 65536 4096 > gpurun_out/stats_base_ff.log 2>&1
TW_LIB=$L/libtimewarp_stats.so timeout -k 10 300 python tools/stats_probe.py 65536 4096 > gpurun_out/stats_new_ff.log 2>&1
