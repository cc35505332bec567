# Kernel-trace stats of the routing microbench: TAG=x LAYERS=3 bash scripts/gpu_ktrace_route.sh
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-ktr}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_route.py --layers ${LAYERS:-3} --iters 5 > $OUT/prof.log 2>&1
python3 - $OUT <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/prof/**/*kernel_stats.csv', recursive=True)[0]
for r in list(csv.DictReader(open(f)))[:25]:
    print(f"{r['Name'][:70]:70s} n={r['Calls']:>4s} avg={float(r['AverageNs'])/1e3:8.1f}us")
PY
