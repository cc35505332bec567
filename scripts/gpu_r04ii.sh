# gux16 peeled capsule loop: DR GPU tests against ab/peel.so, then C4 A/B (alternating).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/r04ii
mkdir -p $OUT
SRF_LIB_PATH=$GRAFT_REPO_ROOT/ab/peel.so timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_route_dr_gpu.py -m gpu > $OUT/pytest.txt 2>&1
rc=$?; tail -3 $OUT/pytest.txt; [ $rc -le 1 ] || exit $rc
TAG=r04ii/c4 VARIANTS="X=0;SRF_LIB_PATH=$GRAFT_REPO_ROOT/ab/peel.so;X=0;SRF_LIB_PATH=$GRAFT_REPO_ROOT/ab/peel.so" timeout -k 10 700 bash scripts/gpu_ab_c4lib.sh
