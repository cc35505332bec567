# Parity of A/B libraries on the GPU suites that cover them, then their kernel timing:
#   TAG=name ABLIBS="ab/x.so ..." TESTS="tests/test_route_dr_gpu.py ..." [LAYERS=c4] bash scripts/gpu_ab_check.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-abcheck}
mkdir -p $OUT
for lib in $ABLIBS; do
  n=$(basename $lib .so)
  SRF_LIB_PATH=$GRAFT_REPO_ROOT/$lib timeout -k 10 600 python -u -m pytest $TESTS -m gpu -x -q --timeout 300 \
    --timeout-method thread > $OUT/pytest_$n.log 2>&1
  rc=$?
  echo "== $n pytest rc=$rc"; tail -3 $OUT/pytest_$n.log
  [ $rc -ne 0 ] && [ $rc -ne 1 ] && exit $rc
done
TAG=${TAG:-abcheck} bash scripts/gpu_ab_route.sh
