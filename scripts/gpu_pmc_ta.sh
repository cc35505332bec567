# TA / TCP counters of the routing microbench (2 TA_ per pass): TAG=x LAYERS=3 bash scripts/gpu_pmc_ta.sh
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pmcta}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
set -e
n=0
for P in "TA_TA_BUSY_sum TA_BUFFER_TOTAL_CYCLES_sum GRBM_GUI_ACTIVE" "TA_ADDR_STALLED_BY_TC_CYCLES_sum TA_DATA_STALLED_BY_TC_CYCLES_sum" "TCP_PENDING_STALL_CYCLES_sum TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCP_TA_DATA_STALL_CYCLES_sum"; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $OUT/p$n -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_route.py --layers ${LAYERS:-3} --iters 3 > $OUT/p$n.log 2>&1
done
python3 $GRAFT_REPO_ROOT/scripts/pmcsum.py $OUT "${FILTER:-route}" 2>&1 | head -120
