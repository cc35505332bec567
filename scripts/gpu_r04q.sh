# C3 A/B of the din-32 SDR contraction kernels (16x16x4 vs 32x32x2 f32 tiles per pose /
# gx / gW; SRF_SDR_MFMA32_DIN32 builds), after the SDR tests on each variant's kernels.
set -o pipefail
cd $GRAFT_REPO_ROOT
for v in 3 6 7; do
  TAG=r04q/t$v TAILN=3 bash scripts/gpu_steps.sh \
    "200|pytest|SRF_LIB_PATH=ab/m32_$v.so python -u -m pytest -q --timeout 100 --timeout-method thread -m gpu tests/test_route_sdr_gpu.py"
  rc=$?
  [ $rc -gt 1 ] && exit $rc
done
TAG=r04q/ab WL=wsj_c3 STEPS=5 VARIANTS="SRF_LIB_PATH=srf_amd/libsrf.so;SRF_LIB_PATH=ab/m32_3.so;SRF_LIB_PATH=ab/m32_6.so;SRF_LIB_PATH=ab/m32_7.so;SRF_LIB_PATH=srf_amd/libsrf.so;SRF_LIB_PATH=ab/m32_3.so;SRF_LIB_PATH=ab/m32_6.so;SRF_LIB_PATH=ab/m32_7.so" bash scripts/gpu_ab_env.sh || exit $?
