# C5 (fp32) bench with A/B builds of libsrf (SRF_LIB_PATH), default build first.
#   LIBS="ab/x.so ab/y.so" TAG=name bash scripts/gpu_lib_ab_c5.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-libab}
mkdir -p $OUT
for lib in default $LIBS; do
  n=$(basename $lib .so)
  if [ $lib = default ]; then unset SRF_LIB_PATH; else export SRF_LIB_PATH=$GRAFT_REPO_ROOT/$lib; fi
  timeout -k 10 300 python -u bench.py --workload ${WL:-wsj_c5} --extra= --no-cpu-baseline --steps 2 --warmup 1 > $OUT/$n.json 2> $OUT/$n.err || { tail -3 $OUT/$n.err; exit 1; }
  python -c "import json; d=json.load(open('$OUT/$n.json')); r=d['roofline']; print('$n', d['ms_per_step'], d['forward_only']['ms_per_step'], r and r['avg_launch_us'])"
done
