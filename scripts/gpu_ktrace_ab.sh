# Kernel-trace stats of the routing microbench for several ab/*.so: TAG=x ALT="a b" LAYERS=3 FILTER=route_acc bash scripts/gpu_ktrace_ab.sh
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-ktrab}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for a in main ${ALT}; do
  if [ "$a" = main ]; then L=$GRAFT_REPO_ROOT/srf_amd/libsrf.so; else L=$GRAFT_REPO_ROOT/ab/$a.so; fi
  SRF_LIB_PATH=$L timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$a -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_route.py --layers ${LAYERS:-3} --iters 5 > $OUT/$a.log 2>&1
  python3 - $OUT/$a "$a" "${FILTER:-route_}" <<'PY'
import csv, glob, sys
f = glob.glob(sys.argv[1] + '/**/*kernel_stats.csv', recursive=True)[0]
for r in csv.DictReader(open(f)):
    if sys.argv[3] in r['Name']:
        print(f"{sys.argv[2]:8s} {r['Name'][:60]:60s} n={r['Calls']:>4s} avg={float(r['AverageNs'])/1e3:8.1f}us")
PY
done
