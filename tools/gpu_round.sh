#!/bin/bash
# One GPU session: each step under its own time limit; stop at the first step
# that aborted, faulted, hung or timed out (exit codes other than 0/1).
# usage: bash tools/gpu_round.sh STEP... (logs under gpurun_out/; the summaries
# worth keeping are copied into profiles/<round><pass>/).  Modifiers between
# steps: geo=G (TW_GEOMETRY), lib=NAME (an A/B build), env=K=V, sfx=S (log
# name suffix).  Rounds 1-3's one-off session scripts are folded into these steps.
export TMPDIR=/tmp
mkdir -p gpurun_out
SFX=""
step() {  # step NAME SECONDS CMD...
  local name=$1$SFX secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "gpurun_out/$name.log" 2>&1
  local rc=$?
  echo "$name=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping after $name (rc=$rc)"; exit $rc; fi
  return 0
}
for s in "$@"; do
  case $s in
    pytest) step pytest_gpu 1000 python -u -m pytest tests/ -q -m gpu -x --timeout 300 --timeout-method thread ;;
    smoke)  step smoke 300 python -c "import __graft_entry__ as g; g.smoke()" ;;
    phase)  step phase 300 python tools/phase_probe.py 65536 4096 ;;
    micro)  step micro 300 python tools/micro_probe.py 65536 8 ;;
    probe)  step probe 300 env TW_LIB=$PWD/time-warp_amd/lib/libtimewarp_prof.so python tools/kernel_probe.py 65536 4096 ;;
    stats) step stats 300 env TW_LIB=$PWD/time-warp_amd/lib/libtimewarp_stats.so python tools/stats_probe.py 65536 4096 ;;
    stats_base) step stats_base 300 env TW_LIB=$PWD/time-warp_amd/lib/libtimewarp_stats_base.so python tools/stats_probe.py 65536 4096 ;;
    stats_c4) step stats_c4 300 env TW_LIB=$PWD/time-warp_amd/lib/libtimewarp_stats.so python -u tools/stats_probe.py gossip ;;
    stats_c5) step stats_c5 400 env TW_LIB=$PWD/time-warp_amd/lib/libtimewarp_stats.so python -u tools/stats_probe.py hotspot 4096 256 ;;
    probe2) step probe2 300 env TW_LIB=$PWD/time-warp_amd/lib/libtimewarp_prof2.so python tools/kernel_probe.py 65536 4096 ;;
    bench)  step bench 500 python bench.py ;;
    tie_c3) step tie_c3 400 python -u tools/ab_probe.py token_ring 65536 auto tie=fifo tie=forkfirst ;;
    tie_c2) step tie_c2 400 python -u tools/ab_probe.py ping_pong 1048576 auto tie=fifo tie=forkfirst ;;
    tie_c3_8k) step tie_c3_8k 400 python -u tools/ab_probe.py token_ring 8192 narrow tie=fifo tie=forkfirst ;;
    benchq) step benchq 300 python bench.py --steps 2 --no-cpu-baseline ;;
    bench_c2) step bench_c2 400 python bench.py --config ping_pong ;;
    bench_c4) step bench_c4 500 python bench.py --config gossip ;;
    benchq_c4) step benchq_c4 300 python bench.py --config gossip --steps 2 --warmup 1 --no-cpu-baseline ;;
    benchq_c4h) step benchq_c4h 300 python bench.py --config gossip --steps 2 --warmup 1 --no-cpu-baseline --host-windows ;;
    prof_c4) step prof_c4 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c4 -o run -- python3 bench.py --config gossip --steps 2 --warmup 1 --no-cpu-baseline ;;
    prof_c3) step prof_c3 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3 -o run -- python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline ;;
    gossip) step gossip 400 python -u -m pytest tests/test_gpu_gossip.py -q -m gpu -x --timeout 120 --timeout-method thread ;;
    bench_msg) step bench_msg 500 python bench.py --duration-s 24576 --drop-log2 16 --steps 2 --warmup 1 ;;
    pmct_msg) PMC_SET=traffic bash tools/pmc_passes.sh gpurun_out/pmct_msg$SFX --duration-s 24576 --drop-log2 16 > gpurun_out/pmct_msg$SFX.log 2>&1; rc=$?; echo "pmct_msg=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    pmc_full) bash tools/pmc.sh gpurun_out/pmc_full > gpurun_out/pmc_full.log 2>&1; rc=$?; echo "pmc_full=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    bench_c5) step bench_c5 400 python bench.py --config hotspot ;;
    benchq_c5) step benchq_c5 400 python bench.py --config hotspot --steps 2 --warmup 1 --no-cpu-baseline ;;
    benchq_c3_8k) step benchq_c3_8k 300 python bench.py --replicas 8192 --steps 2 --warmup 1 --no-cpu-baseline ;;
    benchq_c2) step benchq_c2 300 python bench.py --config ping_pong --steps 2 --warmup 1 --no-cpu-baseline ;;
    geo=*) export TW_GEOMETRY=${s#geo=}; SFX=_${s#geo=} ;;
    env=*) kv=${s#env=}; export "${kv%%=*}=${kv#*=}" ;;
    sfx=*) SFX=_${s#sfx=} ;;
    pytest_geo) step pytest_geo 600 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread -k "$TW_GEOMETRY" ;;
    lib=default) unset TW_LIB; SFX="" ;;
    lib=*) export TW_LIB=$PWD/time-warp_amd/lib/libtimewarp_${s#lib=}.so; SFX=_${s#lib=} ;;
    pmcq_c3_8k) bash tools/pmc_passes.sh gpurun_out/pmcq_c3_8k$SFX --replicas 8192 > gpurun_out/pmcq_c3_8k$SFX.log 2>&1; rc=$?; echo "pmcq_c3_8k=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    pmcq_c3) bash tools/pmc_passes.sh gpurun_out/pmcq_c3$SFX > gpurun_out/pmcq_c3$SFX.log 2>&1; rc=$?; echo "pmcq_c3=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    pmct_c3) PMC_SET=traffic bash tools/pmc_passes.sh gpurun_out/pmct_c3$SFX > gpurun_out/pmct_c3$SFX.log 2>&1; rc=$?; echo "pmct_c3=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    pmcq_c5) bash tools/pmc_passes.sh gpurun_out/pmcq_c5$SFX --config hotspot > gpurun_out/pmcq_c5$SFX.log 2>&1; rc=$?; echo "pmcq_c5=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    calib) mkdir -p gpurun_out/calib && timeout -k 10 120 ./tools/ubench/pmc_calib > gpurun_out/calib/run.log 2>&1 && timeout -s KILL 60 rocprofv3 --pmc FETCH_SIZE --kernel-trace --output-format csv -d gpurun_out/calib/f -o run -- ./tools/ubench/pmc_calib > gpurun_out/calib/f.log 2>&1 && timeout -s KILL 60 rocprofv3 --pmc WRITE_SIZE --kernel-trace --output-format csv -d gpurun_out/calib/w -o run -- ./tools/ubench/pmc_calib > gpurun_out/calib/w.log 2>&1 && python3 tools/pmc_calib.py gpurun_out/calib/pmc_calibration.json gpurun_out/calib/run.log gpurun_out/calib/f gpurun_out/calib/w > gpurun_out/calib/summary.log 2>&1; rc=$?; echo "calib=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    pmc) bash tools/pmc.sh gpurun_out/pmc$SFX > gpurun_out/pmc$SFX.log 2>&1; rc=$?; echo "pmc=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    multi_tests) step multi_tests 400 python -u -m pytest tests/test_gpu_multi.py -x -v --timeout 200 --timeout-method thread ;;
    fusion_tests) step fusion_tests 400 python -u -m pytest tests/test_send_fusion.py -x -q -m gpu --timeout 200 --timeout-method thread ;;
    throw_tests) step throw_tests 300 python -u -m pytest tests/test_gpu_throw_sequences.py -x -q -m gpu --timeout 120 --timeout-method thread ;;
    parity_all) step parity_all 900 python -u tools/parity_all.py c3 c2 c5 ;;
    parity_c3) step parity_c3 600 python -u tools/parity_all.py c3 ;;
    parity_c2c5) step parity_c2c5 900 python -u tools/parity_all.py c2 c5 ;;
    parity_c5) step parity_c5 600 python -u tools/parity_all.py c5 ;;
    lpb_batch_tests) step lpb_batch_tests 600 python -u -m pytest tests/test_gpu_lpb.py -x -v --timeout 300 --timeout-method thread -k "batched" ;;
    lpb_new) step lpb_new 600 python -u -m pytest tests/test_gpu_lpb.py -x -v --timeout 300 --timeout-method thread -k "benched_shape_256 or over_the_cap or full_lane" ;;
    core_tests) step core_tests 900 python -u -m pytest tests/test_gpu_programs.py tests/test_gpu_tie_orders.py tests/test_gpu_parity.py tests/test_gpu_throw_sequences.py -x -q -m gpu --timeout 300 --timeout-method thread ;;
    ab_c3) bash tools/ab_session.sh token_ring; rc=$?; echo "ab_c3=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    lpb_tests) step lpb_tests 500 python -u -m pytest tests/test_gpu_lpb.py -x -v --timeout 200 --timeout-method thread ;;
    stats_c3_lpb) step stats_c3_lpb 400 env TW_LIB=$PWD/time-warp_amd/lib/libtimewarp_stats.so python -u tools/stats_probe.py lpb_token 8192 ;;
    stats_c5_lpb) step stats_c5_lpb 400 env TW_LIB=$PWD/time-warp_amd/lib/libtimewarp_stats.so python -u tools/stats_probe.py lpb_hotspot 4096 256 ;;
    prof_c5) step prof_c5 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c5 -o run -- python3 bench.py --config hotspot --steps 1 --warmup 0 --no-cpu-baseline ;;
    prof_c3_8k_lpb) step prof_c3_8k_lpb 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_c3_8k_lpb -o run -- python3 bench.py --replicas 8192 --geometry lpb --steps 1 --warmup 0 --no-cpu-baseline ;;
    bench_c3_8k) step bench_c3_8k 400 python bench.py --replicas 8192 ;;
    benchq_c3_32k) step benchq_c3_32k 300 python bench.py --replicas 32768 --steps 2 --warmup 1 --no-cpu-baseline ;;
    benchq_c3_16k) step benchq_c3_16k 300 python bench.py --replicas 16384 --steps 2 --warmup 1 --no-cpu-baseline ;;
    benchq_c3_32k_lpb) step benchq_c3_32k_lpb 400 python bench.py --replicas 32768 --geometry lpb --steps 1 --warmup 1 --no-cpu-baseline ;;
    benchq_c3_16k_lpb) step benchq_c3_16k_lpb 300 python bench.py --replicas 16384 --geometry lpb --steps 2 --warmup 1 --no-cpu-baseline ;;
    benchq_c3_8k_lpb) step benchq_c3_8k_lpb 300 python bench.py --replicas 8192 --geometry lpb --steps 2 --warmup 1 --no-cpu-baseline ;;
    pmct_c5) bash tools/pmc_traffic.sh gpurun_out/pmct_c5$SFX --config hotspot > gpurun_out/pmct_c5$SFX.log 2>&1; rc=$?; echo "pmct_c5=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    pmct_c2) bash tools/pmc_traffic.sh gpurun_out/pmct_c2$SFX --config ping_pong > gpurun_out/pmct_c2$SFX.log 2>&1; rc=$?; echo "pmct_c2=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    pmct_c4) bash tools/pmc_traffic.sh gpurun_out/pmct_c4$SFX --config gossip > gpurun_out/pmct_c4$SFX.log 2>&1; rc=$?; echo "pmct_c4=$rc"; [ $rc -eq 0 ] || exit $rc ;;
    # A/B of an alternative build (lib=NAME -> time-warp_amd/lib/libtimewarp_NAME.so) is
    # a sequence like: lib=old benchq_c5 benchq_c4 lib=default benchq_c5 benchq_c4
    *) echo "unknown step $s"; exit 2 ;;
  esac
done
