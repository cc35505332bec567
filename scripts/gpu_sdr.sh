# SDR recurrence check on the GPU box: parity tests (new + legacy kernels), the SDR
# model fixture, then the C3 bench with the register-resident kernels and the legacy ones.
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-sdr}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_route_sdr_gpu.py tests/test_model_gpu.py -x -v --timeout 120 --timeout-method thread > $OUT/pytest.log 2>&1 || { tail -40 $OUT/pytest.log; exit 1; }
tail -3 $OUT/pytest.log
timeout -k 10 300 python bench.py --workload wsj_c3 --steps 5 --warmup 2 --no-cpu-baseline > $OUT/bench_c3.json 2> $OUT/bench_c3.err
cat $OUT/bench_c3.json
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload wsj_c3 --steps 3 --warmup 1 --no-cpu-baseline > $OUT/prof.log 2>&1
ls -R $OUT | head -20
