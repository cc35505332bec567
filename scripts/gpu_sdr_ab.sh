# Timing A/B of the SDR recurrence kernels: C3 bench kernel traces with the in-tree
# library and the timing-experiment builds under build/dbg*/.
set -e
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-sdrab}
mkdir -p $OUT
cd /tmp && export TMPDIR=/tmp
for v in main ${ALT}; do
  if [ $v = main ]; then L=$GRAFT_REPO_ROOT/srf_amd/libsrf.so; else L=$GRAFT_REPO_ROOT/build/$v/libsrf.so; fi
  SRF_LIB_PATH=$L timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d $OUT/$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --workload wsj_c3 --steps 2 --warmup 1 --no-cpu-baseline > $OUT/$v.log 2>&1
done
ls $OUT
