# PMC passes (separate runs, kernel-trace only) on a command: CMD env (default: routing microbench layer 3).
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pmc}
mkdir -p $OUT
CMD=${CMD:-"python3 $GRAFT_REPO_ROOT/scripts/bench_route.py --layers 3 --iters 3"}
cd /tmp && export TMPDIR=/tmp
timeout -k 10 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
set -e
n=0
for P in "SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_INSTS_VALU SQ_INSTS_MFMA" \
         "SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_INSTS_VMEM_WR SQ_INSTS_VMEM_RD SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_SALU" \
         "FETCH_SIZE" "WRITE_SIZE" "TCC_HIT_sum TCC_MISS_sum"; do
  n=$((n+1))
  timeout -k 10 240 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $OUT/p$n -o run -- $CMD > $OUT/p$n.log 2>&1
done
ls -R $OUT | head -40
