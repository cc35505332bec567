# C5 fp8 A/B (raw bf16 ring slots) and a C5 kernel-trace profile of the A/B lib.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04ee
mkdir -p $OUT
WL=wsj_c5_fp8 LIBS="ab/slot.so" TAG=r04ee/c5fp8 timeout -k 10 700 bash scripts/gpu_lib_ab_c5.sh || exit $?
cd /tmp && export TMPDIR=/tmp
SRF_LIB_PATH=$GRAFT_REPO_ROOT/ab/slot.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload wsj_c5 --extra= --no-cpu-baseline --steps 1 --warmup 1 > $OUT/prof.log 2>&1 || { tail -5 $OUT/prof.log; exit 1; }
f=$(find $OUT/prof -name '*kernel_stats.csv' | head -1); cp $f $OUT/kernel_stats_c5.csv
python3 - $OUT/kernel_stats_c5.csv <<'PY'
import csv, sys
for r in list(csv.DictReader(open(sys.argv[1])))[:14]:
    print(f"{r['Name'][:90]:90s} n={r['Calls']:>5s} tot={float(r['TotalDurationNs'])/1e6:8.1f}ms avg={float(r['AverageNs'])/1e3:9.1f}us {r['Percentage']}")
PY
