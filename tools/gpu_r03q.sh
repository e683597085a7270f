# round-3 GPU session Q: is C5's window the receiver's chain?  senders 64/128/256 at fewer messages
export TMPDIR=/tmp
O=gpurun_out/r03q
mkdir -p $O
for S in 64 128 256; do
  timeout -k 10 300 python3 -u bench.py --config hotspot --nodes $S --msg-num 200 --steps 1 --warmup 1 --no-cpu-baseline > $O/c5_s$S.log 2>&1; rc=$?; echo "s$S=$rc"
  [ $rc -eq 0 ] || exit $rc
done
timeout -k 10 300 python3 -u bench.py --config hotspot --replicas 1024 --msg-num 200 --steps 1 --warmup 1 --no-cpu-baseline > $O/c5_r1024.log 2>&1; rc=$?; echo "r1024=$rc"
exit $rc
