# Kernel-level A/B of the DR routing layer at the C4 bench size (B = 28, T' = 200):
# rocprofv3 kernel statistics of scripts/bench_route.py for the shipped library and
# each library in ABLIBS (timing builds may compute wrong results: they are only timed).
#   TAG=name [LAYERS=c4,c4last] ABLIBS="ab/x.so ab/y.so" bash scripts/gpu_ab_route.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-abroute}
LAYERS=${LAYERS:-c4}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for lib in base $ABLIBS; do
  n=$(basename $lib .so)
  if [ "$lib" = base ]; then unset SRF_LIB_PATH; else export SRF_LIB_PATH=$GRAFT_REPO_ROOT/$lib; fi
  timeout -k 10 150 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o run -- \
    python3 $GRAFT_REPO_ROOT/scripts/bench_route.py --layers $LAYERS --B 28 --T 200 --iters 10 > $OUT/$n.log 2>&1 \
    || { tail -5 $OUT/$n.log; exit 1; }
  echo "== $n"; grep "layer" $OUT/$n.log | tail -2; grep "blk" $OUT/$n.log | head -8 || true
  python3 $GRAFT_REPO_ROOT/scripts/kstats.py $OUT/$n/run_kernel_stats.csv 13 12
done
