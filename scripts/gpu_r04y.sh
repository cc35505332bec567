# Fused SDR gx + gW on bf16 MFMA with three-term split operands: tests, then C3 A/B
# against the f32-MFMA fused kernel (ab/gxwf32.so).
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r04y TAILN=6 bash scripts/gpu_steps.sh \
  "400|pytest|python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_route_sdr_gpu.py tests/test_model_gpu.py tests/test_parity_scale_gpu.py -k 'sdr or c3 or pose or fused'"
rc=$?
[ $rc -gt 1 ] && exit $rc
TAG=r04y/ab WL=wsj_c3 STEPS=5 VARIANTS="SRF_LIB_PATH=ab/gxwf32.so;SRF_LIB_PATH=srf_amd/libsrf.so;SRF_LIB_PATH=ab/gxwf32.so;SRF_LIB_PATH=srf_amd/libsrf.so" bash scripts/gpu_ab_env.sh || exit $?
exit $rc
