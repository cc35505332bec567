# SDR stack range-size A/B on C3 (SRF_SDR_CHUNKS ranges per utterance; default 10 = 20 frames).
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-chunks}
mkdir -p $OUT
for c in ${CHUNKS:-10 14 20}; do
  SRF_SDR_CHUNKS=$c timeout -k 10 300 python -u bench.py --workload wsj_c3 --extra= --no-cpu-baseline --steps 10 --warmup 2 > $OUT/c3_k$c.json 2> $OUT/c3_k$c.err || { tail -3 $OUT/c3_k$c.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/c3_k$c.json')); print('chunks $c', d['ms_per_step'], d['forward_only']['ms_per_step'])"
done
