# Parity tests of the in-tree library (TESTS), then bench A/B against ab/*.so (ALT = names):
#   TAG=x ALT="base" TESTS="tests/test_route_dr_gpu.py" bash scripts/gpu_libab.sh
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-libab}
mkdir -p $OUT
if [ -n "${TESTS}" ]; then
timeout -k 10 400 python -u -m pytest ${TESTS} -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
fi
for rep in 1 2; do
for v in main ${ALT}; do
  if [ "$v" = main ]; then L=""; else L="SRF_LIB_PATH=$GRAFT_REPO_ROOT/ab/$v.so"; fi
  env $L timeout -k 10 200 python bench.py --no-cpu-baseline --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS} > $OUT/$v.$rep.json 2> $OUT/$v.$rep.err
  python3 -c "import json,sys; d=json.load(open('$OUT/$v.$rep.json')); print('$v', d['ms_per_step'], d['roofline']['avg_launch_us'] if d.get('roofline') else '')"
done
done
if [ -n "${ROUTE}" ]; then
for v in main ${ALT}; do
  if [ "$v" = main ]; then L=""; else L="SRF_LIB_PATH=$GRAFT_REPO_ROOT/ab/$v.so"; fi
  echo "$v"; env $L timeout -k 10 120 python scripts/bench_route.py --layers ${ROUTE} --iters 20 2>/dev/null
done
fi
