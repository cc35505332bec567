# Fused SDR gx/gW workgroup size A/B (16 / 8 / 4 waves): its parity test per build, then C3.
set -o pipefail
cd $GRAFT_REPO_ROOT
for lib in ab/gxw8.so ab/gxw4.so; do
  n=$(basename $lib .so)
  TAG=r04w/$n TAILN=3 bash scripts/gpu_steps.sh \
    "200|pytest|SRF_LIB_PATH=$lib python -u -m pytest -q --timeout 100 --timeout-method thread -m gpu tests/test_route_sdr_gpu.py -k fused"
  rc=$?
  [ $rc -ne 0 ] && exit $rc
done
TAG=r04w/ab WL=wsj_c3 STEPS=5 VARIANTS="SRF_LIB_PATH=srf_amd/libsrf.so;SRF_LIB_PATH=ab/gxw8.so;SRF_LIB_PATH=ab/gxw4.so;SRF_LIB_PATH=srf_amd/libsrf.so;SRF_LIB_PATH=ab/gxw8.so;SRF_LIB_PATH=ab/gxw4.so" bash scripts/gpu_ab_env.sh || exit $?
