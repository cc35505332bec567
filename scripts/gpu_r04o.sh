# SDR tests on the shipped library (backward group 2 by default on the C3 last layer),
# per-frame G = 1, 2 times of both gu-pass variants, then a C3 A/B.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r04o
mkdir -p $OUT
TAG=r04o TAILN=4 bash scripts/gpu_steps.sh \
  "300|pytest|python -u -m pytest -q --timeout 200 --timeout-method thread -m gpu tests/test_route_sdr_gpu.py tests/test_model_gpu.py -k 'sdr or c3'"
rc=$?
[ $rc -gt 1 ] && exit $rc
for lib in srf_amd/libsrf.so ab/gr1.so; do
  n=$(basename $lib .so)
  SDR_GROUPS=1,2 SRF_LIB_PATH=$lib timeout -k 10 120 python3 -u scripts/sdr_group_frames.py > $OUT/groups_$n.log 2>&1 || { tail -5 $OUT/groups_$n.log; exit 1; }
  echo "[$lib]"; grep -v amdgpu.ids $OUT/groups_$n.log
done
TAG=r04o/ab WL=wsj_c3 STEPS=5 VARIANTS="SRF_LIB_PATH=srf_amd/libsrf.so;SRF_LIB_PATH=ab/gr1.so;SRF_LIB_PATH=srf_amd/libsrf.so;SRF_LIB_PATH=ab/gr1.so;SRF_LIB_PATH=srf_amd/libsrf.so --sdr-last-group=1" bash scripts/gpu_ab_env.sh || exit $?
exit $rc
