# GPU parity suite + smoke + default bench line.
#   TAG=name [PYTEST_ARGS=...] [BENCH_ARGS=...] [NO_BENCH=1] bash scripts/gpu_check.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-check}
mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/ -m gpu -v --timeout 300 --timeout-method thread ${PYTEST_ARGS} ${PYTEST_K:+-k "$PYTEST_K"} \
  > $OUT/pytest.log 2>&1
rc=$?
tail -30 $OUT/pytest.log
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi      # 1 = failures (read the log), else crash/timeout
timeout -k 10 180 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || { cat $OUT/smoke.log; exit 3; }
cat $OUT/smoke.log
if [ -z "$NO_BENCH" ]; then
  timeout -k 10 600 python -u bench.py ${BENCH_ARGS} > $OUT/bench.json 2> $OUT/bench.err || { tail -30 $OUT/bench.err; exit 4; }
  cat $OUT/bench.json
fi
exit $rc
