# device-drawn link tables: their GPU tests, the fusion tests again, a C3 bench line with the device draw
export TMPDIR=/tmp
O=gpurun_out/r03tb
mkdir -p $O
run() {  # run NAME SECONDS CMD...
  local name=$1 secs=$2; shift 2
  timeout -k 10 "$secs" "$@" > "$O/$name.log" 2>&1
  local rc=$?
  echo "$name=$rc"
  [ $rc -eq 0 ] || exit $rc
}
run tables 400 python -u -m pytest tests/test_gpu_tables.py tests/test_abi.py -x -v -s -m "gpu or not gpu" --timeout 300 --timeout-method thread
run bq_c3 400 python3 bench.py --steps 2 --warmup 1 --no-cpu-baseline
run bq_c3_host 400 python3 bench.py --steps 1 --warmup 0 --no-cpu-baseline --host-tables
exit 0
