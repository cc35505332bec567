# C3 recurrence kernel A/B: register-resident (default) vs streaming for the J=32 last
# layer (SRF_SDR_SEQ_MAXJD=512) or every layer (SRF_SDR_SEQ=0).  TAG=name bash scripts/gpu_sdr_ab2.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-sdrab2}
mkdir -p $OUT
run() {  # name env...
  local n=$1; shift
  timeout -k 10 300 env "$@" python -u bench.py --workload wsj_c3 --extra= --no-cpu-baseline --steps 10 --warmup 2 > $OUT/$n.json 2> $OUT/$n.err || exit 1
  python -c "import json; d=json.load(open('$OUT/$n.json')); print('$n', d['ms_per_step'], d['forward_only']['ms_per_step'])"
}
run c3_base SRF_NOTHING=1
run c3_last_stream SRF_SDR_SEQ_MAXJD=512
run c3_all_stream SRF_SDR_SEQ=0
