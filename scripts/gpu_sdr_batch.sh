# SDR stack: parity tests, then C3 / C5 benches with the batched diagonals (default)
# and the per-layer streams (SRF_SDR_BATCH=0).   TAG=name bash scripts/gpu_sdr_batch.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-sdrbatch}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_model_gpu.py tests/test_route_sdr_gpu.py -q --timeout 200 --timeout-method thread \
  -k "sdr or c3 or c5" > $OUT/pytest.log 2>&1
rc=$?; tail -5 $OUT/pytest.log
if [ $rc -ne 0 ]; then grep -E "FAILED|Error" $OUT/pytest.log | head -20; exit $rc; fi
run() {  # name steps workload env...
  local n=$1 st=$2 wl=$3; shift 3
  timeout -k 10 300 env "$@" python -u bench.py --workload $wl --extra= --no-cpu-baseline --steps $st --warmup 2 > $OUT/$n.json 2> $OUT/$n.err || { tail -5 $OUT/$n.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$n.json')); print('$n', d['ms_per_step'], d['forward_only']['ms_per_step'])"
}
run c3_batch 10 wsj_c3 SRF_X=1
run c3_perlayer 10 wsj_c3 SRF_SDR_BATCH=0
run c5_batch 2 wsj_c5 SRF_X=1
