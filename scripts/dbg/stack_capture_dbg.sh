set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/s2n
timeout -k 10 200 python -u bench.py --workload wsj_c3 --extra= --no-cpu-baseline --steps 3 --warmup 2 --eager > gpurun_out/s2n/eager.json 2> gpurun_out/s2n/eager.err; echo "eager rc=$?"
tail -3 gpurun_out/s2n/eager.err
AMD_LOG_LEVEL=1 timeout -k 10 200 python -u bench.py --workload wsj_c3 --extra= --no-cpu-baseline --steps 3 --warmup 2 > gpurun_out/s2n/graph.json 2> gpurun_out/s2n/graph.err; echo "graph rc=$?"
tail -c 3000 gpurun_out/s2n/graph.err
