# A/B timings (no parity) of the routing microbench for each library build under ab/.
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-ab}
mkdir -p $OUT
set -e
for L in ab/*.so; do
  n=$(basename $L .so)
  (cd /tmp && TMPDIR=/tmp SRF_LIB_PATH=$GRAFT_REPO_ROOT/$L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/$n -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_route.py --layers ${LAYERS:-3} --iters 5 > $OUT/$n.log 2>&1)
done
