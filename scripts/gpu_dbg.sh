# Kernel timings of the routing microbench under SRF_DBG experiment knobs.
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-dbg}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
set -e
for D in ${DBGS:-0 1 2 4 8}; do
  SRF_DBG=$D timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/d$D -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_route.py --layers ${LAYERS:-3} --iters 5 > $OUT/d$D.log 2>&1
done
