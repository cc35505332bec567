# TA/TCP/TCC counters of the routing microbenchmark: TAG=x LAYERS="c4 --B 28 --T 200" bash scripts/gpu_pmc_ta2.sh
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pmcta2}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
set -e
n=0
for P in "TA_BUSY_avr TA_ADDR_STALLED_BY_TC_CYCLES_sum GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_INSTS_VALU SQ_INSTS_MFMA SQ_INSTS_LDS SQ_WAVE_CYCLES" "TCP_TCC_READ_REQ_sum TCP_TOTAL_CACHE_ACCESSES_sum TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE"; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $OUT/p$n -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_route.py --layers ${LAYERS:-3} --iters 3 > $OUT/p$n.log 2>&1
done
python3 $GRAFT_REPO_ROOT/scripts/pmcsum.py $OUT 2>&1 | head -120
