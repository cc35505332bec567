# SDR forward with the next frame's loads in flight across the barriers (unconditional,
# raw barriers) and three of five rows staged through LDS on the C3 inner layers:
# SDR / model tests, per-frame times, then a C3 A/B against ab/nostage.so.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04aa
mkdir -p $OUT
TAG=r04aa TAILN=6 bash scripts/gpu_steps.sh \
  "400|pytest|python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_route_sdr_gpu.py tests/test_model_gpu.py tests/test_parity_scale_gpu.py -k 'sdr or c3'"
rc=$?
[ $rc -gt 1 ] && exit $rc
for lib in srf_amd/libsrf.so ab/nostage.so; do
  n=$(basename $lib .so)
  SDR_GROUPS=1 SRF_LIB_PATH=$lib timeout -k 10 120 python3 -u scripts/sdr_group_frames.py > $OUT/frames_$n.log 2>&1 || { tail -5 $OUT/frames_$n.log; exit 1; }
  echo "[$lib]"; grep -v amdgpu.ids $OUT/frames_$n.log
done
TAG=r04aa/ab WL=wsj_c3 STEPS=5 VARIANTS="SRF_LIB_PATH=ab/nostage.so;SRF_LIB_PATH=srf_amd/libsrf.so;SRF_LIB_PATH=ab/nostage.so;SRF_LIB_PATH=srf_amd/libsrf.so" bash scripts/gpu_ab_env.sh || exit $?
exit $rc
