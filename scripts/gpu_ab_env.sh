# A/B of environment settings / bench flags on one bench workload, one process per variant.
#   TAG=name WL=wsj_c3 VARIANTS="A=1 --flag=2;A=0" [STEPS=5] bash scripts/gpu_ab_env.sh
# (words of a variant starting with -- go to bench.py, the others into its environment)
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-abenv}
mkdir -p $OUT
IFS=';' read -ra VS <<< "$VARIANTS"
i=0
for v in "${VS[@]}"; do
  i=$((i+1))
  envs=(); args=()
  for w in $v; do
    if [[ $w == --* ]]; then args+=("$w"); else envs+=("$w"); fi
  done
  env "${envs[@]}" timeout -k 10 ${VTLIM:-300} python -u bench.py --workload ${WL:-wsj_c3} --extra= --no-cpu-baseline \
    --steps ${STEPS:-5} --warmup 2 "${args[@]}" > $OUT/v$i.json 2> $OUT/v$i.err || { echo "variant [$v] failed"; tail -5 $OUT/v$i.err; exit 1; }
  python -c "import json,sys; d=json.load(open('$OUT/v$i.json')); r=d['roofline'] or {}; print('[$v]', d['ms_per_step'], 'ms', d['forward_only']['ms_per_step'], 'fwd ms', r.get('avg_launch_us'), 'us', r.get('frac'))"
done
