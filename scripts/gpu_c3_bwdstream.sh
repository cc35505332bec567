# C3: streaming backward for the register-path layers (SRF_SDR_BWD_STREAM=1) vs default;
# parity of the stack with it first.   TAG=name bash scripts/gpu_c3_bwdstream.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-c3bs}
mkdir -p $OUT
SRF_SDR_BWD_STREAM=1 timeout -k 10 300 python -u -m pytest tests/test_model_gpu.py -q --timeout 200 --timeout-method thread -k "c3" > $OUT/pytest.log 2>&1
rc=$?; tail -3 $OUT/pytest.log; [ $rc -ne 0 ] && exit $rc
for x in ${XS:-1 0 1 0}; do
  SRF_SDR_BWD_STREAM=$x timeout -k 10 300 python -u bench.py --workload wsj_c3 --extra= --no-cpu-baseline --steps 10 --warmup 2 > $OUT/c3_$x.json 2> $OUT/c3_$x.err || { tail -3 $OUT/c3_$x.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/c3_$x.json')); print('bwd_stream=$x', d['ms_per_step'])"
done
