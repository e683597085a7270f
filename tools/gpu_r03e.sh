# round-3 GPU session E: every config on the fixed engine, plus the compact geometry on C3
export TMPDIR=/tmp
O=gpurun_out/r03e
mkdir -p $O
run() {  # name, args...
  n=$1; shift
  timeout -k 10 300 python -u bench.py --steps 3 --warmup 1 --no-cpu-baseline "$@" > $O/$n.log 2>&1; rc=$?; echo "$n=$rc"
  [ $rc -eq 0 ] || exit $rc
}
run c3_dense
run c3_compact --geometry compact
run c3_8k_narrow --replicas 8192
run c3_8k_compact --replicas 8192 --geometry compact
run c2 --config ping_pong
run c4 --config gossip
run c5 --config hotspot
