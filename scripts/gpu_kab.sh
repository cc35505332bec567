# Kernel-trace A/B of environment variants on the routing microbenchmark:
#   TAG=x LAYERS=c4 BT="--B 28 --T 200" VARS="A=1 A=2,B=3" bash scripts/gpu_kab.sh
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-kab}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in base ${VARS}; do
  n=$(echo $v | tr '/=,' '___')
  envs=$(echo $v | tr ',' ' ')
  [ "$v" = base ] && envs="X=1"
  env $envs timeout -k 10 200 python3 $GRAFT_REPO_ROOT/scripts/bench_route.py --layers ${LAYERS:-c4} --iters 10 ${BT} > $OUT/$n.txt 2>&1
  cat $OUT/$n.txt
  export $envs
  timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/$n -o run -- python3 $GRAFT_REPO_ROOT/scripts/bench_route.py --layers ${LAYERS:-c4} --iters 10 ${BT} > $OUT/$n.prof.log 2>&1
  unset $(echo $envs | sed 's/=[^ ]*//g')
  python3 $GRAFT_REPO_ROOT/scripts/kstats.py $OUT/$n/run_kernel_stats.csv 13 ${TOPK:-10}
done
