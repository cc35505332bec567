# Kernel timings (no parity) for each library under ab/: TAG=x FILTER=route_fwd32 LAYERS=1,3 bash scripts/gpu_abk.sh
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-abk}
mkdir -p $OUT
set -e
for rep in 1 2; do for L in ab/*.so; do
  n=$(basename $L .so)
  (cd /tmp && TMPDIR=/tmp SRF_LIB_PATH=$GRAFT_REPO_ROOT/$L timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/$n$rep -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_route.py --layers ${LAYERS:-1,3} --iters 5 > $OUT/$n$rep.log 2>&1)
  echo "== $n"; grep layer $OUT/$n$rep.log
  python3 scripts/ktrace.py $(ls $OUT/$n$rep/*/run_kernel_trace.csv $OUT/$n$rep/run_kernel_trace.csv 2>/dev/null | head -1) "${FILTER:-route}" | head -${TOPN:-12}
done; done
