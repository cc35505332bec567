# split-fp16 gradient passes: parity tests, C4 env A/B (one process per variant),
# kernel stats.   TAG=name [VARIANTS=...] bash scripts/gpu_gux16.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-gux16}
mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_route_dr_gpu.py -x -q --timeout 200 --timeout-method thread \
  > $OUT/pytest_dr.log 2>&1; rc=$?
tail -5 $OUT/pytest_dr.log
if [ $rc -ne 0 ]; then echo "pytest rc=$rc"; exit $rc; fi
TAG=${TAG:-gux16}/ab WL=${WL:-wsj_c4} STEPS=20 VARIANTS="${VARIANTS:-SRF_GW16=1;SRF_GW16=0;SRF_GW16=1;SRF_GW16=0 SRF_GUX16=0}" \
  bash scripts/gpu_ab_env.sh || exit 1
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/prof -o run -- python3 \
  $GRAFT_REPO_ROOT/bench.py --workload ${WL:-wsj_c4} --extra= --no-cpu-baseline --steps 10 --warmup 3 > $OUT/prof.log 2>&1 \
  || { tail -5 $OUT/prof.log; exit 1; }
find $OUT/prof -name "*kernel_stats.csv" | head -1 | xargs -I{} cp {} $OUT/kernel_stats.csv
python3 $GRAFT_REPO_ROOT/scripts/kstats.py $OUT/kernel_stats.csv 2>/dev/null | head -20 || head -12 $OUT/kernel_stats.csv | cut -c1-150
