# Kernel-trace of graphed training steps: TAG=name WL=timit_c2 bash scripts/gpu_stepprof.sh
set -e
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-sp}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for W in ${WL:-timit_c2}; do
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/$W -o run -- python3 $GRAFT_REPO_ROOT/scripts/stepprof.py $W ${STEPS:-10} > $OUT/$W.log 2>&1
python3 $GRAFT_REPO_ROOT/scripts/stepbreak.py $(ls $OUT/$W/*/run_kernel_trace.csv $OUT/$W/run_kernel_trace.csv 2>/dev/null | head -1) ${STEPS:-10} > $OUT/$W.break.txt
head -50 $OUT/$W.break.txt
done
