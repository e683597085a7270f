# round-3 GPU session U: per-pass cost in the replica geometries (dense / narrow) for comparison with lpb
export TMPDIR=/tmp
O=gpurun_out/r03u
mkdir -p $O
timeout -k 10 300 python3 -u tools/pass_probe.py 64 16384 50 dense > $O/pass_dense.log 2>&1; rc=$?; echo "dense=$rc"
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python3 -u tools/pass_probe.py 64 4096 50 narrow > $O/pass_narrow.log 2>&1; rc=$?; echo "narrow=$rc"
exit $rc
