# C5 (L=8 DIM=64 LPAD=RPAD=20 SDR iter=5) bench line, eager, 2 timed steps.
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-c5}
mkdir -p $OUT
timeout -k 10 500 python -u bench.py --workload wsj_c5 --steps 2 --warmup 1 --eager --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail -20 $OUT/bench_c5.err; exit 1; }
cat $OUT/bench_c5.json
