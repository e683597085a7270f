export TMPDIR=/tmp
mkdir -p gpurun_out/geo
for R in 32768 16384; do
  for G in narrow dense; do
    TW_GEOMETRY=$G timeout -k 10 300 python bench.py --replicas $R --steps 2 --warmup 1 --no-cpu-baseline > gpurun_out/geo/c3_${R}_$G.log 2>&1; rc=$?; echo "c3_${R}_$G=$rc"
    [ $rc -eq 0 ] || exit $rc
  done
done
