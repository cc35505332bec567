# Issue/wait breakdown (SQ counters, one --pmc pass each) of one bench workload, plus
# an env A/B of the same workload.  TAG=name WL=wsj_c4 AB="SRF_LIB_PATH=ab/x.so" [PENV="A=1 B=2"] bash scripts/gpu_pmc_sq2.sh
# (PENV: environment of the profiled runs)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pmcsq2}
mkdir -p $OUT/sq
B="$GRAFT_REPO_ROOT/bench.py --workload ${WL:-wsj_c4} --extra= --no-cpu-baseline"
if [ -n "$AB" ]; then
  for rep in 1 2; do
    timeout -k 10 300 python3 -u $B --steps 20 --warmup 5 > $OUT/ab_base_$rep.json 2> $OUT/ab_base_$rep.err || exit 1
    timeout -k 10 300 env $AB python3 -u $B --steps 20 --warmup 5 > $OUT/ab_var_$rep.json 2> $OUT/ab_var_$rep.err || exit 1
  done
fi
cd /tmp && export TMPDIR=/tmp
timeout -s KILL 60 rocprofv3 -L > $OUT/sq/avail.txt 2>&1 || true
n=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU SQ_INSTS_MFMA SQ_WAIT_INST_LDS" "SQ_INSTS_SALU SQ_INSTS_LDS SQ_INSTS_VMEM_RD SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_MISC SQ_INST_CYCLES_SALU SQ_ACTIVE_INST_LDS SQ_WAVES"; do
  n=$((n+1))
  env $PENV timeout -s KILL 200 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $OUT/sq/p$n -o run -- python3 $B --steps 2 --warmup 1 \
    > $OUT/sq/p$n.log 2>&1 || { tail -5 $OUT/sq/p$n.log; echo "pass $n failed"; }
done
echo done
