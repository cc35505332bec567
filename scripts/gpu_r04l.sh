# Round-4 SDR check: SDR tests, then (only if pytest neither crashed nor timed out) the
# C3 profile and a C3 library A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r04l TAILN=8 bash scripts/gpu_steps.sh \
  "300|pytest|python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_route_sdr_gpu.py tests/test_model_gpu.py -k 'sdr or c3'"
rc=$?
[ $rc -gt 1 ] && exit $rc
TAG=r04l ABLIBS=ab/base.so bash scripts/gpu_c3prof.sh || exit $?
TAG=r04l/ab WL=wsj_c3 STEPS=5 VARIANTS="SRF_LIB_PATH=srf_amd/libsrf.so;SRF_LIB_PATH=ab/base.so;SRF_LIB_PATH=srf_amd/libsrf.so;SRF_LIB_PATH=ab/base.so" bash scripts/gpu_ab_env.sh || exit $?
exit $rc
