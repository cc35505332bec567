# Routing-layer iteration on the GPU box: parity tests of the routing layers,
# microbench (default path and SRF_ROUTE_FWD32=0), optional full bench.
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-route}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_route_dr_gpu.py ${EXTRA_TESTS} -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python scripts/bench_route.py --layers ${LAYERS:-1,3} --chunks 0 2>&1 | tee $OUT/route.txt
SRF_ROUTE_FWD32=0 timeout -k 10 300 python scripts/bench_route.py --layers ${LAYERS:-1,3} --chunks 0 2>&1 | tee $OUT/route_old.txt
if [ -n "$BENCH" ]; then
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/bench.json 2> $OUT/bench.err
cat $OUT/bench.json
fi
