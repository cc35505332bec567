# Selected GPU tests in one process.   TAG=name PYTEST_ARGS="tests/x.py -k y" bash scripts/gpu_pytest.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-pytest}
mkdir -p $OUT
timeout -k 10 ${TLIM:-900} python -u -m pytest -x -v --timeout 300 --timeout-method thread -m gpu ${PYTEST_ARGS:-tests/} \
  > $OUT/pytest.log 2>&1
rc=$?
tail -40 $OUT/pytest.log
exit $rc
