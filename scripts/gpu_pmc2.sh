# Memory-hierarchy PMC passes of the routing microbench: FETCH_SIZE, L2 hit/miss, L1.
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pmc2}
mkdir -p $OUT
CMD="python3 $GRAFT_REPO_ROOT/scripts/bench_route.py --layers ${LAYERS:-3} --iters 3"
cd /tmp && export TMPDIR=/tmp
n=0
for P in "FETCH_SIZE" "TCC_HIT_sum TCC_MISS_sum" "TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum" "TA_BUSY_avr TA_TA_BUSY_sum" ; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $OUT/p$n -o run -- $CMD > $OUT/p$n.log 2>&1 || echo "pass $n failed: $P"
done
ls $OUT
