# C2 bench step time for forced fwd32 i-chunk counts (0 = auto).
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-f32c}
mkdir -p $OUT
for c in 0 2 3 4 6 8 12; do
  SRF_FWD32_CHUNKS=$c timeout -k 10 200 python bench.py --no-cpu-baseline > $OUT/c$c.json 2> $OUT/c$c.err
  python -c "import json; d=json.load(open('$OUT/c$c.json')); print('chunks $c', d['ms_per_step'], d['roofline']['avg_launch_us'])"
done
