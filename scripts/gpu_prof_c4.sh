# Kernel-trace stats of the C4 bench.  Usage: TAG=name bash scripts/gpu_prof_c4.sh
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-profc4}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload wsj_c4 --steps 3 --warmup 1 --eager --no-cpu-baseline > $OUT/prof.log 2>&1
tail -1 $OUT/prof.log
