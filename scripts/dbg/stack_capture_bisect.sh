# Graph-captured C3 step under the SDR stack's optional overlaps (bisection of a capture crash).
#   A=<gw_stream> P=<pose_ahead> bash scripts/dbg/stack_capture_bisect.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bisect
for cfg in $CFGS; do
  g=${cfg%,*}; p=${cfg#*,}
  SRF_SDR_GW_STREAM=$g SRF_SDR_POSE_AHEAD=$p timeout -k 10 200 python -u bench.py --workload wsj_c3 --extra= --no-cpu-baseline --steps 5 --warmup 2 > gpurun_out/bisect/g${g}p${p}.json 2> gpurun_out/bisect/g${g}p${p}.err
  rc=$?; echo "gw_stream=$g pose_ahead=$p rc=$rc"; tail -c 400 gpurun_out/bisect/g${g}p${p}.err
  [ $rc -ne 0 ] && exit $rc
  python -c "import json; d=json.load(open('gpurun_out/bisect/g${g}p${p}.json')); print(d['ms_per_step'])"
done
