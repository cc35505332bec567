# Iteration run on the GPU box: parity tests, routing microbench, bench line, kernel stats.
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-iter}
mkdir -p $OUT
timeout -k 10 400 python -m pytest tests/ -m gpu -q -x 2>&1 | tail -8
timeout -k 10 300 python scripts/bench_route.py --layers ${LAYERS:-1,3} --chunks 0 2>&1 | tee $OUT/route.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1
ls $OUT/prof
