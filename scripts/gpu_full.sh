# Round evidence run on the GPU box: parity tests, smoke, bench lines (C2 with CPU
# baseline, C4, C3), kernel-trace stats of the C2 bench, FETCH/WRITE PMC passes.
# Usage: TAG=name bash scripts/gpu_full.sh
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-full}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/ -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -30 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
cat $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench_c2.json 2> $OUT/bench_c2.err
cat $OUT/bench_c2.json
if [ -z "$SKIP_WSJ" ]; then
timeout -k 10 300 python bench.py --workload wsj_c4 --steps 10 --warmup 3 --no-cpu-baseline > $OUT/bench_c4.json 2> $OUT/bench_c4.err
cat $OUT/bench_c4.json
timeout -k 10 300 python bench.py --workload wsj_c3 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err
cat $OUT/bench_c3.json
fi
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1
n=0
for P in FETCH_SIZE WRITE_SIZE; do
  n=$((n+1))
  timeout -s KILL 120 rocprofv3 --kernel-trace --pmc $P --output-format csv -d $OUT/p$n -o run -- python3 $GRAFT_REPO_ROOT/bench.py --steps 3 --warmup 1 --no-cpu-baseline > $OUT/p$n.log 2>&1
done
ls -R $OUT | head -30
