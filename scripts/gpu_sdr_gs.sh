# SDR parity tests, then the C5 bench line.  Usage: TAG=name bash scripts/gpu_sdr_gs.sh
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-sdrgs}
mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_route_sdr_gpu.py tests/test_model_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -60 $OUT/pytest.log; exit 1; }
tail -2 $OUT/pytest.log
timeout -k 10 500 python -u bench.py --workload wsj_c5 --steps 2 --warmup 1 --eager --no-cpu-baseline > $OUT/bench_c5.json 2> $OUT/bench_c5.err || { tail -20 $OUT/bench_c5.err; exit 1; }
cat $OUT/bench_c5.json
