# Iteration run: routing + model GPU tests, then the routing microbench under a kernel trace.
# TAG=x [LAYERS=1,3] [TESTS="tests/test_route_dr_gpu.py tests/test_model_gpu.py"] bash scripts/gpu_iter.sh
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-iter}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest ${TESTS:-tests/test_route_dr_gpu.py tests/test_model_gpu.py} -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
cd /tmp && export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace --output-format csv -d $OUT/tr -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_route.py --layers ${LAYERS:-1,3} --iters 5 > $OUT/route.log 2>&1
grep layer $OUT/route.log
python3 $GRAFT_REPO_ROOT/scripts/ktrace.py $(ls $OUT/tr/*/run_kernel_trace.csv $OUT/tr/run_kernel_trace.csv 2>/dev/null | head -1) "${FILTER:-}" > $OUT/ktrace.txt; head -${TOPN:-16} $OUT/ktrace.txt
