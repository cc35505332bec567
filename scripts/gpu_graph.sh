# hipGraph train step check: all GPU tests, then the C2 bench graphed and eager.
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-graph}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_graph.json 2> $OUT/bench_graph.err || { tail -20 $OUT/bench_graph.err; exit 1; }
cat $OUT/bench_graph.json
timeout -k 10 300 python bench.py --no-cpu-baseline --eager > $OUT/bench_eager.json 2> $OUT/bench_eager.err
cat $OUT/bench_eager.json
timeout -k 10 300 python bench.py --no-cpu-baseline --workload wsj_c3 --steps 5 --warmup 2 > $OUT/bench_c3.json 2> $OUT/bench_c3.err
cat $OUT/bench_c3.json
