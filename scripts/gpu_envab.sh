# Parity tests (TESTS), then bench A/B of environment settings (VARS, each "A=1,B=2") and ab/*.so (ALT):
#   TAG=x VARS="SRF_FWD32_SPLIT=0" ALT="head" TESTS="tests/test_route_dr_gpu.py" ROUTE=1,3 bash scripts/gpu_envab.sh
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-envab}
mkdir -p $OUT
if [ -n "${TESTS}" ]; then
timeout -k 10 400 python -u -m pytest ${TESTS} -m gpu -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
fi
run() {  # name env...
  n=$1; shift
  env "$@" timeout -k 10 200 python bench.py --no-cpu-baseline --steps ${STEPS:-20} --warmup 5 ${BENCH_ARGS} > $OUT/$n.json 2> $OUT/$n.err
  python3 -c "import json,sys; d=json.load(open('$OUT/$n.json')); print('$n', d['ms_per_step'], d['roofline']['avg_launch_us'] if d.get('roofline') else '')"
  if [ -n "${ROUTE}" ]; then env "$@" timeout -k 10 120 python scripts/bench_route.py --layers ${ROUTE} --iters 20 2>/dev/null; fi
}
for rep in 1 2; do
  run main.$rep X=1
  for v in ${VARS}; do run $(echo $v | tr '/=,' '___').$rep $(echo $v | tr ',' ' '); done
  for a in ${ALT}; do run $a.$rep SRF_LIB_PATH=$GRAFT_REPO_ROOT/ab/$a.so; done
done
