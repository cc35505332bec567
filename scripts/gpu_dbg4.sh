# s_memtime phase breakdown of route_fwd32_kernel (ab/dbg4.so built with -DSRF_FWD32_DBG=4): TAG=x LAYERS=1,3 bash scripts/gpu_dbg4.sh
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-dbg4}
mkdir -p $OUT
SRF_LIB_PATH=$GRAFT_REPO_ROOT/ab/dbg4.so timeout -k 10 120 python scripts/bench_route.py --layers ${LAYERS:-1,3} --iters 2 > $OUT/dbg4.txt 2>&1
grep "fwd32 NW" $OUT/dbg4.txt | sort | uniq | head -16
