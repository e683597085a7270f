mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 bench.py --config hotspot --steps 1 --warmup 0 --no-cpu-baseline > gpurun_out/prof_c5.log 2>&1
rc=$?
echo "prof rc=$rc"
[ $rc -eq 0 ] || exit $rc
python3 - <<'PY'
import json,sys,glob
import os
TW=os.path.join(os.getcwd(),'time-warp_amd')
sys.path.insert(0,TW)
PY
TW_LIB=$PWD/time-warp_amd/lib/libtimewarp.so timeout -k 10 300 python3 -c "
import sys; sys.path.insert(0,'time-warp_amd')
from timewarp import scenarios
from timewarp.engine import Engine, draw_link_table
scn = scenarios.hotspot(n_senders=256, n_replicas=4096, msg_num=1000, drawer=draw_link_table)
with Engine(0) as e:
    e.load(scn, geometry='lpb')
    e.reset(); st = e.run()
    print('events', st.events, 'kernel_ms', st.kernel_ms, 'windows', e.lpb_windows(), 'batch', e.lpb_batch())
" > gpurun_out/c5_batchstats.log 2>&1
