# SDR register backward: LDS-only barriers and the frame's rows loaded right after its
# couplings (in flight to the adjoint): SDR / model tests, per-frame times, C3 A/B
# against ab/bwdold.so.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04bb
mkdir -p $OUT
TAG=r04bb TAILN=6 bash scripts/gpu_steps.sh \
  "400|pytest|python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_route_sdr_gpu.py tests/test_model_gpu.py tests/test_parity_scale_gpu.py -k 'sdr or c3'"
rc=$?
[ $rc -gt 1 ] && exit $rc
for lib in srf_amd/libsrf.so ab/bwdold.so; do
  n=$(basename $lib .so)
  SDR_GROUPS=1,2 SRF_LIB_PATH=$lib timeout -k 10 120 python3 -u scripts/sdr_group_frames.py > $OUT/frames_$n.log 2>&1 || { tail -5 $OUT/frames_$n.log; exit 1; }
  echo "[$lib]"; grep -v amdgpu.ids $OUT/frames_$n.log
done
TAG=r04bb/ab WL=wsj_c3 STEPS=5 VARIANTS="SRF_LIB_PATH=ab/bwdold.so;SRF_LIB_PATH=srf_amd/libsrf.so;SRF_LIB_PATH=ab/bwdold.so;SRF_LIB_PATH=srf_amd/libsrf.so" bash scripts/gpu_ab_env.sh || exit $?
exit $rc
