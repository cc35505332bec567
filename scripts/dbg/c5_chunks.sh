set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/s2u
mkdir -p $OUT
for c in 20 10; do
  SRF_SDR_CHUNKS=$c timeout -k 10 300 python -u bench.py --workload wsj_c5 --extra= --no-cpu-baseline --steps 2 --warmup 1 > $OUT/c5_k$c.json 2> $OUT/c5_k$c.err || { tail -3 $OUT/c5_k$c.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/c5_k$c.json')); print('c5 chunks $c', d['ms_per_step'], d['forward_only']['ms_per_step'])"
done
