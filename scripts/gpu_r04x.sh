# fp32 SDR pose on bf16 MFMA with three-term split operands: accuracy test and SDR /
# model suites, then C3 and C5 against the 32x32x2 f32 pose (ab/posef32.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r04x TAILN=6 bash scripts/gpu_steps.sh \
  "400|pytest|python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_route_sdr_gpu.py tests/test_model_gpu.py tests/test_parity_scale_gpu.py -k 'sdr or c3 or c5 or pose'"
rc=$?
[ $rc -gt 1 ] && exit $rc
TAG=r04x/ab WL=wsj_c3 STEPS=5 VARIANTS="SRF_LIB_PATH=ab/posef32.so;SRF_LIB_PATH=srf_amd/libsrf.so;SRF_LIB_PATH=ab/posef32.so;SRF_LIB_PATH=srf_amd/libsrf.so" bash scripts/gpu_ab_env.sh || exit $?
TAG=r04x/ab5 WL=wsj_c5 STEPS=2 VTLIM=400 VARIANTS="SRF_LIB_PATH=ab/posef32.so;SRF_LIB_PATH=srf_amd/libsrf.so" bash scripts/gpu_ab_env.sh || exit $?
exit $rc
