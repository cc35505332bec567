# Fused SDR gx + gW (din 32): its parity test and the SDR suites, then a C3 A/B against
# the separate launches.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r04r TAILN=6 bash scripts/gpu_steps.sh \
  "300|pytest|python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_route_sdr_gpu.py tests/test_model_gpu.py -k 'sdr or c3 or fused'"
rc=$?
[ $rc -gt 1 ] && exit $rc
TAG=r04r/ab WL=wsj_c3 STEPS=5 VARIANTS="--sdr-separate-gxgw;SRF_X=1;--sdr-separate-gxgw;SRF_X=1" bash scripts/gpu_ab_env.sh || exit $?
exit $rc
