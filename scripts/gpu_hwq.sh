# A/B of GPU_MAX_HW_QUEUES (HIP hardware queues per process) on the SDR stack benches,
# plus a kernel trace of C5 forward-only at the largest setting (queue ids per stream).
#   TAG=name bash scripts/gpu_hwq.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-hwq}
mkdir -p $OUT
for q in 4 16 32; do
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --workload wsj_c3 --extra= --no-cpu-baseline --steps 10 --warmup 2 > $OUT/c3_q$q.json 2> $OUT/c3_q$q.err || exit 1
  GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python -u bench.py --workload wsj_c5 --extra= --no-cpu-baseline --steps 2 --warmup 1 > $OUT/c5_q$q.json 2> $OUT/c5_q$q.err || exit 2
  python -c "
import json
for w in ('c3', 'c5'):
    d = json.load(open('$OUT/%s_q$q.json' % w)); print('q$q', w, d['ms_per_step'], d['forward_only']['ms_per_step'])"
done
