# A/B of the routing microbench: the in-tree library against build/$ALT/libsrf.so.
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-ab}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_route_dr_gpu.py -x -q --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
for rep in 1 2; do
echo "main" ; timeout -k 10 120 python scripts/bench_route.py --layers ${LAYERS:-1,3} --iters 20 2>/dev/null
for alt in ${ALT}; do echo "$alt"; SRF_LIB_PATH=$GRAFT_REPO_ROOT/build/$alt/libsrf.so timeout -k 10 120 python scripts/bench_route.py --layers ${LAYERS:-1,3} --iters 20 2>/dev/null; done
done
