#!/bin/bash
# A/B session on one box: time-warp_amd/lib/libtimewarp_base.so (the previous
# engine) against libtimewarp.so, alternating; usage: bash tools/ab_session.sh [CONFIG...]
# (CONFIG: a bench.py --config value; default token_ring).  Summary lines go to
# gpurun_out/ab_summary.txt.
mkdir -p gpurun_out
L=$PWD/time-warp_amd/lib
cfgs=${*:-token_ring}
for cfg in $cfgs; do
  for v in base new base new; do
    if [ $v = base ]; then export TW_LIB=$L/libtimewarp_base.so; else export TW_LIB=$L/libtimewarp.so; fi
    timeout -k 10 300 python bench.py --config $cfg --steps 3 --warmup 1 --no-cpu-baseline > gpurun_out/ab_${cfg}_$v.log 2>&1
    rc=$?
    echo "$cfg $v rc=$rc $(grep -o '"ms_per_step": [0-9.]*' gpurun_out/ab_${cfg}_$v.log)" >> gpurun_out/ab_summary.txt
    if [ $rc -ne 0 ]; then exit $rc; fi
  done
done
unset TW_LIB
