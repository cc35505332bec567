set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-r2}
mkdir -p $OUT
timeout -k 10 400 python -m pytest tests/ -m gpu -q -x 2>&1 | tail -8
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 10 > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $OUT/prof.log 2>&1
find $OUT/prof -name "*stats*"
