# GPU tests, smoke, C2 and C4 bench lines.  Usage: TAG=name bash scripts/gpu_ab_xt.sh
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-abxt}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/ -m gpu -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py --no-cpu-baseline > $OUT/bench_c2.json 2> $OUT/bench_c2.err || { tail -20 $OUT/bench_c2.err; exit 1; }
timeout -k 10 300 python bench.py --no-cpu-baseline --workload wsj_c4 --steps 10 --warmup 3 > $OUT/bench_c4.json 2> $OUT/bench_c4.err
for f in bench_c2 bench_c4; do python -c "import json; d=json.load(open('$OUT/$f.json')); print('$f', d['ms_per_step'], d['value'])"; done
