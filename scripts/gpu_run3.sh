set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r3}
mkdir -p $OUT
timeout -k 10 400 python -m pytest tests/ -m gpu -q -x 2>&1 | tail -5
timeout -k 10 300 python scripts/bench_route.py --layers 1,3 --chunks 0,1,2,3,4,6,8,12 2>&1 | tee $OUT/route.txt
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
