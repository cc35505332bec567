# Round-4 SDR backward gu-pass A/B: per-frame times (G = 1, 2), the SDR tests on the
# shipped library, then the C3 step per library.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04m
mkdir -p $OUT
for lib in srf_amd/libsrf.so ab/gr1.so ab/hd8.so; do
  n=$(basename $lib .so)
  GROUPS=1,2 SRF_LIB_PATH=$lib timeout -k 10 120 python3 -u scripts/sdr_group_frames.py > $OUT/groups_$n.log 2>&1 || { tail -5 $OUT/groups_$n.log; exit 1; }
  echo "[$lib]"; grep -v amdgpu.ids $OUT/groups_$n.log
done
TAG=r04m TAILN=4 bash scripts/gpu_steps.sh \
  "300|pytest|python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_route_sdr_gpu.py tests/test_model_gpu.py -k 'sdr or c3'"
rc=$?
[ $rc -gt 1 ] && exit $rc
TAG=r04m/ab WL=wsj_c3 STEPS=5 VARIANTS="SRF_LIB_PATH=srf_amd/libsrf.so;SRF_LIB_PATH=ab/gr1.so;SRF_LIB_PATH=ab/hd8.so;SRF_LIB_PATH=srf_amd/libsrf.so;SRF_LIB_PATH=ab/gr1.so;SRF_LIB_PATH=ab/hd8.so" bash scripts/gpu_ab_env.sh || exit $?
exit $rc
