# SQ counters of the routing microbench: TAG=x LAYERS=3 bash scripts/gpu_pmc_route.sh
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pmcr}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
set -e
n=0
for P in "SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_ACTIVE_INST_VALU SQ_BUSY_CYCLES SQ_WAVES" "GRBM_GUI_ACTIVE GRBM_COUNT SQ_VALU_MFMA_COEXEC_CYCLES SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS"; do
  n=$((n+1))
  SRF_LIB_PATH=${LIB:-$GRAFT_REPO_ROOT/srf_amd/libsrf.so} timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $OUT/p$n -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_route.py --layers ${LAYERS:-3} --iters 3 > $OUT/p$n.log 2>&1
done
python3 $GRAFT_REPO_ROOT/scripts/pmcsum.py $OUT 2>&1 | head -80
[ -n "$LIST" ] && timeout -s KILL 60 rocprofv3 -L > $OUT/counters.txt 2>&1 || true
