# Kernel trace of one workload's eager forward-only passes (the SDR stack timeline).
#   TAG=name WL=wsj_c5 [HWQ=16] bash scripts/gpu_trace_fwd.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-trace}
WL=${WL:-wsj_c5}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
[ -n "$HWQ" ] && export GPU_MAX_HW_QUEUES=$HWQ
timeout -k 10 400 rocprofv3 --kernel-trace --output-format csv -d $OUT/kt_$WL -o run -- \
  python3 $GRAFT_REPO_ROOT/bench.py --workload $WL --extra= --no-cpu-baseline --steps 1 --warmup 1 > $OUT/kt_$WL.log 2>&1 || { tail -20 $OUT/kt_$WL.log; exit 1; }
tail -1 $OUT/kt_$WL.log | cut -c1-200
