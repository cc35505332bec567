# C3 (SDR) bench + kernel stats under environment variants: TAG=x VARS="A=1 B=0" bash scripts/gpu_c3ab.sh
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-c3ab}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in base ${VARS}; do
  n=$(echo $v | tr '/=,' '___'); envs=$(echo $v | tr ',' ' '); [ "$v" = base ] && envs="X=1"
  export $envs
  timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/$n -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload wsj_c3 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/$n.json 2> $OUT/$n.err
  unset $(echo $envs | sed 's/=[^ ]*//g')
  python3 -c "import json; d=json.load(open('$OUT/$n.json')); print('$n', d['ms_per_step'])"
  python3 $GRAFT_REPO_ROOT/scripts/ktrace.py $OUT/$n/run_kernel_trace.csv sdr | head -12
done
