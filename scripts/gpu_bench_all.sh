# Bench lines of every workload: default (C4 headline + C2 extra [+ CPU baseline]),
# C3 and C5.   TAG=name [CPU=1] bash scripts/gpu_bench_all.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-benchall}
mkdir -p $OUT
CB=--no-cpu-baseline
[ -n "$CPU" ] && CB=
timeout -k 10 400 python -u bench.py $CB > $OUT/bench.json 2> $OUT/bench.err || { tail -5 $OUT/bench.err; exit 1; }
timeout -k 10 300 python -u bench.py --workload wsj_c3 --extra= --no-cpu-baseline --steps 10 --warmup 2 \
  > $OUT/c3.json 2> $OUT/c3.err || { tail -5 $OUT/c3.err; exit 2; }
timeout -k 10 600 python -u bench.py --workload wsj_c5 --extra= --no-cpu-baseline --steps 2 --warmup 1 \
  > $OUT/c5.json 2> $OUT/c5.err || { tail -5 $OUT/c5.err; exit 3; }
python - <<PY
import json
d = json.load(open('$OUT/bench.json'))
print('C4', d['value'], d['ms_per_step'], 'frac', d['roofline']['frac'], 'traffic', d['roofline']['traffic'])
e = d['extra']['timit_c2']
print('C2', e['value'], e['ms_per_step'], 'frac', e['roofline']['frac'], 'traffic', e['roofline']['traffic'])
for w in ('c3', 'c5'):
    d = json.load(open('$OUT/%s.json' % w))
    print(w, d['value'], d['ms_per_step'], 'fwd', d['forward_only']['ms_per_step'])
PY
