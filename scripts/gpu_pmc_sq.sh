# LDS bank-conflict and wait counters of one bench workload (one --pmc pass each).
#   TAG=name WL=wsj_c4 bash scripts/gpu_pmc_sq.sh ; then python scripts/pmcsum.py gpurun_out/TAG/sq FILTER
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pmcsq}/sq
mkdir -p $OUT
B="$GRAFT_REPO_ROOT/bench.py --workload ${WL:-wsj_c4} --extra= --no-cpu-baseline --steps 2 --warmup 1"
cd /tmp && export TMPDIR=/tmp
n=0
for P in "SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" "SQ_WAIT_INST_ANY SQ_WAVE_CYCLES"; do
  n=$((n+1))
  timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $OUT/p$n -o run -- python3 $B \
    > $OUT/p$n.log 2>&1 || { tail -5 $OUT/p$n.log; exit 1; }
done
echo done
