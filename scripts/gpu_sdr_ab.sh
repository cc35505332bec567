# SDR stack launch-mode A/B: hipGraph vs eager, HIP hardware queues 4 vs 16.
#   TAG=name bash scripts/gpu_sdr_ab.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-sdrab}
mkdir -p $OUT
run() {  # name steps workload extra-args...
  local n=$1 st=$2 wl=$3; shift 3
  timeout -k 10 300 env "$@" python -u bench.py --workload $wl --extra= --no-cpu-baseline --steps $st --warmup 2 $EAGER > $OUT/$n.json 2> $OUT/$n.err || exit 1
  python -c "import json; d=json.load(open('$OUT/$n.json')); print('$n', d['ms_per_step'], d['forward_only']['ms_per_step'])"
}
EAGER=--eager run c3_eager_q4 10 wsj_c3 GPU_MAX_HW_QUEUES=4
EAGER=--eager run c3_eager_q16 10 wsj_c3 GPU_MAX_HW_QUEUES=16
EAGER= run c3_graph_q16 10 wsj_c3 GPU_MAX_HW_QUEUES=16
EAGER=--eager run c5_eager_q16 2 wsj_c5 GPU_MAX_HW_QUEUES=16
