# Timing variants of the fwd32 pass (build/dbgN/libsrf.so, see SRF_FWD32_DBG).
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-dbg32}
mkdir -p $OUT
echo base > $OUT/dbg.txt
timeout -k 10 120 python scripts/bench_route.py --layers ${LAYERS:-3} --iters 10 2>/dev/null >> $OUT/dbg.txt
for d in 1 2 3; do
  echo "dbg$d" >> $OUT/dbg.txt
  SRF_LIB_PATH=$GRAFT_REPO_ROOT/build/dbg$d/libsrf.so timeout -k 10 120 python scripts/bench_route.py --layers ${LAYERS:-3} --iters 10 2>/dev/null >> $OUT/dbg.txt
done
cat $OUT/dbg.txt
