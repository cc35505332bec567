# Round-end evidence in one call: full GPU suite, smoke, bench lines, C4 / C3 / C2 kernel stats.
#   TAG=name bash scripts/gpu_final.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${TAG:-final}
OUT=$GRAFT_REPO_ROOT/gpurun_out/$T
mkdir -p $OUT
TAILN=4 TAG=$T bash scripts/gpu_steps.sh \
  '900|pytest|python -u -m pytest tests/ -m gpu -v --timeout 300 --timeout-method thread' \
  '240|smoke|python -u -c "import __graft_entry__ as g; g.smoke(); print(\"smoke ok\")"' \
  '400|bench|python -u bench.py' \
  '300|c3|python -u bench.py --workload wsj_c3 --extra= --no-cpu-baseline --steps 10 --warmup 2' \
  '400|c5|python -u bench.py --workload wsj_c5 --extra= --no-cpu-baseline --steps 2 --warmup 1' \
  '400|c5fp8|python -u bench.py --workload wsj_c5_fp8 --extra= --no-cpu-baseline --steps 2 --warmup 1' || exit $?
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 \
  $GRAFT_REPO_ROOT/bench.py --workload wsj_c4 --extra= --no-cpu-baseline --steps 10 --warmup 3 > $OUT/prof.log 2>&1 \
  || { tail -5 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats_c4.csv
for wl in wsj_c3:c3 timit_c2:c2; do
  w=${wl%%:*}; k=${wl##*:}
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof_$k -o run -- python3 \
    $GRAFT_REPO_ROOT/bench.py --workload $w --extra= --no-cpu-baseline --steps 6 --warmup 2 > $OUT/prof_$k.log 2>&1 \
    || { tail -5 $OUT/prof_$k.log; exit 1; }
  find $OUT/prof_$k -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats_$k.csv
done

cd $GRAFT_REPO_ROOT
