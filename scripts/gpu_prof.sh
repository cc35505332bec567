# Profile of one bench workload: kernel-trace statistics, then (PMC=1) the FETCH_SIZE and
# WRITE_SIZE passes and (SQ=1) two SQ issue / wait passes -- each --pmc pass a run of
# its own, within the per-block counter limits.
#   TAG=name WL=wsj_c4 [STEPS=10] [PMC=1] [SQ=1] bash scripts/gpu_prof.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-prof}
WL=${WL:-wsj_c4}
STEPS=${STEPS:-10}
mkdir -p $OUT
B="$GRAFT_REPO_ROOT/bench.py --workload $WL --extra= --no-cpu-baseline"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt_$WL -o run -- \
  python3 $B --steps $STEPS --warmup 2 > $OUT/kt_$WL.log 2>&1 || { tail -20 $OUT/kt_$WL.log; exit 1; }
tail -1 $OUT/kt_$WL.log
PASSES=()
[ -n "$PMC" ] && PASSES+=("FETCH_SIZE" "WRITE_SIZE")
[ -n "$SQ" ] && PASSES+=(
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS"
  "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAVES")
n=0
for P in "${PASSES[@]}"; do
  n=$((n+1))
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $OUT/pmc_${WL}/p$n -o run -- \
    python3 $B --steps 2 --warmup 1 > $OUT/pmc_${WL}_p$n.log 2>&1 || { tail -20 $OUT/pmc_${WL}_p$n.log; echo "pass $n failed"; exit 2; }
done
echo done
