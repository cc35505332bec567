# A/B: parity of the routing tests and kernel timings for each library build under ab/.
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-ab}
mkdir -p $OUT
set -e
for L in ab/*.so; do
  n=$(basename $L .so)
  SRF_LIB_PATH=$GRAFT_REPO_ROOT/$L timeout -k 10 200 python -m pytest -q -x tests/test_route_dr_gpu.py 2>&1 | tail -1
  (cd /tmp && TMPDIR=/tmp SRF_LIB_PATH=$GRAFT_REPO_ROOT/$L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/$n -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_route.py --layers ${LAYERS:-1,3} --iters 5 > $OUT/$n.log 2>&1)
  grep layer $OUT/$n.log
done
