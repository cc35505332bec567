# Bench A/B by environment: TAG=x VARS="A=1 B=2" bash scripts/gpu_benchab.sh  (each VAR runs as its own bench)
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-benchab}
mkdir -p $OUT
for rep in 1 2; do
for v in base ${VARS}; do
  if [ "$v" = base ]; then e=""; else e="$v"; fi
  n=$(echo "$v" | tr '/=' '__')
  env $e timeout -k 10 200 python bench.py --no-cpu-baseline --steps ${STEPS:-20} --warmup 5 > $OUT/$n.$rep.json 2> $OUT/$n.$rep.err
  python3 -c "import json,sys; d=json.load(open('$OUT/$n.$rep.json')); print('$v', d['ms_per_step'], d['roofline']['avg_launch_us'] if d.get('roofline') else '')"
done
done
