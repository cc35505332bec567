# B1 passes: logZ loaded ahead and the next capsule's loads / pose unconditional, so the
# stores no longer wait for the prefetch: DR / model / parity tests, then a C4 A/B
# against ab/b1old.so.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r04cc TAILN=6 bash scripts/gpu_steps.sh \
  "400|pytest|python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_route_dr_gpu.py tests/test_model_gpu.py tests/test_parity_scale_gpu.py"
rc=$?
[ $rc -gt 1 ] && exit $rc
TAG=r04cc/ab WL=wsj_c4 STEPS=20 VARIANTS="SRF_LIB_PATH=ab/b1old.so;SRF_LIB_PATH=srf_amd/libsrf.so;SRF_LIB_PATH=ab/b1old.so;SRF_LIB_PATH=srf_amd/libsrf.so;SRF_LIB_PATH=ab/b1old.so;SRF_LIB_PATH=srf_amd/libsrf.so" bash scripts/gpu_ab_env.sh || exit $?
exit $rc
