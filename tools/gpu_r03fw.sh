# ADDI+Jcc pairs fused, hot in the LP kernels only: its GPU tests, the whole GPU suite, quick bench lines for C2..C5
export TMPDIR=/tmp
O=gpurun_out/r03fw
mkdir -p $O
run() {  # run NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name=$rc"
  [ $rc -eq 0 ] || exit $rc
}
run fusion 300 python -u -m pytest tests/test_send_fusion.py -x -v -m gpu --timeout 120 --timeout-method thread
run pytest_gpu 700 python -u -m pytest tests/ -q -m gpu -x --timeout 120 --timeout-method thread
run bq_c4 300 python3 bench.py --config gossip --steps 2 --warmup 1 --no-cpu-baseline
run bq_c5 300 python3 bench.py --config hotspot --steps 2 --warmup 1 --no-cpu-baseline
run bq_c2 300 python3 bench.py --config ping_pong --steps 2 --warmup 1 --no-cpu-baseline
run bq_c3 300 python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline
run bq_c3_8k 300 python3 bench.py --replicas 8192 --steps 2 --warmup 1 --no-cpu-baseline
exit 0
