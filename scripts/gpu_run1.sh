set -e
cd $GRAFT_REPO_ROOT
timeout -k 10 400 python -m pytest tests/test_route_dr_gpu.py tests/test_model_gpu.py -q -x 2>&1 | tail -15
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --cpu-seconds 10 > gpurun_out/bench1.json 2> gpurun_out/bench1.err
cat gpurun_out/bench1.json
cd /tmp && export TMPDIR=/tmp && timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $GRAFT_REPO_ROOT/gpurun_out/prof1 -o run -- python $GRAFT_REPO_ROOT/bench.py --steps 10 --warmup 3 --no-cpu-baseline > $GRAFT_REPO_ROOT/gpurun_out/prof1.log 2>&1
ls -R $GRAFT_REPO_ROOT/gpurun_out/prof1 | head
