# Batched capsnorm ranges in the SDR stack: SDR / model tests, then a C3 A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r04s TAILN=6 bash scripts/gpu_steps.sh \
  "300|pytest|python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_route_sdr_gpu.py tests/test_model_gpu.py tests/test_caps_gpu.py -k 'sdr or c3 or caps or norm'"
rc=$?
[ $rc -gt 1 ] && exit $rc
TAG=r04s/ab WL=wsj_c3 STEPS=5 VARIANTS="--sdr-capsnorm-per-layer;SRF_X=1;--sdr-capsnorm-per-layer;SRF_X=1" bash scripts/gpu_ab_env.sh || exit $?
exit $rc
