# Sweep SRF_FWD32_CHUNKS for the routing microbench (layer ${LAYERS:-3}).
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-chunks}
mkdir -p $OUT
for c in ${CHUNKS:-0 2 3 4 5 6 8 12}; do
  echo "chunks=$c" >> $OUT/sweep.txt
  SRF_FWD32_CHUNKS=$c timeout -k 10 120 python scripts/bench_route.py --layers ${LAYERS:-3} --chunks 0 --iters 10 2>/dev/null >> $OUT/sweep.txt
done
cat $OUT/sweep.txt
