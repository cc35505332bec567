# Kernel-trace stats and FETCH/WRITE PMC passes of one bench workload.
#   TAG=name WL=wsj_c4 [STEPS=10] [PMC=1] bash scripts/gpu_prof.sh
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
if [ -n "$PMC" ]; then
  n=0
  for P in FETCH_SIZE WRITE_SIZE; do
    n=$((n+1))
    timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $OUT/pmc_${WL}_$n -o run -- \
      python3 $B --steps 2 --warmup 1 > $OUT/pmc_${WL}_$n.log 2>&1 || { tail -20 $OUT/pmc_${WL}_$n.log; exit 2; }
  done
fi
ls -R $OUT | head -40
