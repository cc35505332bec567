# DR parity tests, then C4 A/B over (library, env) variants.
#   TAG=name VARIANTS="..." bash scripts/gpu_split16_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-split16}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_route_dr_gpu.py -x -q --timeout 200 --timeout-method thread \
  > $OUT/pytest_dr.log 2>&1; rc=$?
tail -3 $OUT/pytest_dr.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
TAG=${TAG:-split16}/ab WL=${WL:-wsj_c4} STEPS=20 bash scripts/gpu_ab_env.sh
