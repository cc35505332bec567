# Round-4 profile of the C4 step: kernel-trace statistics, FETCH/WRITE PMC passes and
# two SQ issue/wait passes (each --pmc pass a run of its own), plus the fp8 pose dump.
#   TAG=name [WL=wsj_c4] bash scripts/gpu_prof_r04.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-prof04}
WL=${WL:-wsj_c4}
mkdir -p $OUT
timeout -k 10 120 python3 -u scripts/dbg/fp8_pose_dump.py $OUT/fp8_pose_dump.npz > $OUT/fp8.log 2>&1 || { tail -5 $OUT/fp8.log; exit 1; }
B="$GRAFT_REPO_ROOT/bench.py --workload $WL --extra= --no-cpu-baseline"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 400 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- \
  python3 $B --steps 10 --warmup 2 > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
tail -1 $OUT/kt.log
n=0
for P in "FETCH_SIZE" "WRITE_SIZE" \
  "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS" \
  "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_BUSY_CYCLES SQ_ACTIVE_INST_LDS SQ_WAVES"; do
  n=$((n+1))
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $OUT/pmc/p$n -o run -- \
    python3 $B --steps 2 --warmup 1 > $OUT/pmc_p$n.log 2>&1 || { tail -5 $OUT/pmc_p$n.log; echo "pass $n failed"; exit 2; }
done
echo done
