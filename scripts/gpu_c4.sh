# din-32 DR check: route parity tests, then C4 (and C2) bench lines and C4 kernel stats.
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-c4}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_route_dr_gpu.py} -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 300 python bench.py --workload wsj_c4 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_c4.json 2> $OUT/bench_c4.err
cat $OUT/bench_c4.json


timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err
cat $OUT/bench_c2.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload wsj_c4 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/prof.log 2>&1
