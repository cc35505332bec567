# C3 kernel trace after the round-4 stack changes, and the C5 / C5 fp8 bench lines.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04t
mkdir -p $OUT
timeout -k 10 400 python -u bench.py --workload wsj_c5 --extra= --no-cpu-baseline --steps 2 --warmup 1 > $OUT/c5.json 2> $OUT/c5.err || { tail -5 $OUT/c5.err; exit 1; }
tail -c 400 $OUT/c5.json
B="$GRAFT_REPO_ROOT/bench.py --workload wsj_c3 --extra= --no-cpu-baseline"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- \
  python3 $B --steps 5 --warmup 2 > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
tail -1 $OUT/kt.log | cut -c1-300
