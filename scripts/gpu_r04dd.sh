# Stream-kernel A/B: SDR GPU tests against the A/B lib, then C5 default vs A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04dd
mkdir -p $OUT
SRF_LIB_PATH=$GRAFT_REPO_ROOT/ab/ldsbar.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_route_sdr_gpu.py -m gpu > $OUT/pytest.txt 2>&1
rc=$?; tail -3 $OUT/pytest.txt; [ $rc -le 1 ] || exit $rc
LIBS="ab/ldsbar.so" TAG=r04dd/c5 timeout -k 10 700 bash scripts/gpu_lib_ab_c5.sh
