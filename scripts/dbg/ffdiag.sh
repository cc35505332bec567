# Kernel traces of the iteration-0 GEMM in three builds (main, and ab/ffd1.so / ab/ffd2.so
# built with -DSRF_FF_DIAG=1 (no DMA after capsule 0) / =2 (DMA only, no fragment reads or
# MFMAs) on a temporary copy of route_fwd32.hip's loop): bash scripts/dbg/ffdiag.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/r06o
cd /tmp && export TMPDIR=/tmp
for v in main ffd1 ffd2; do
  if [ $v = main ]; then L=$GRAFT_REPO_ROOT/srf_amd/libsrf.so; else L=$GRAFT_REPO_ROOT/ab/$v.so; fi
  SRF_LIB_PATH=$L timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d $GRAFT_REPO_ROOT/gpurun_out/r06o/$v -o run -- python3 $GRAFT_REPO_ROOT/bench.py --extra= --no-cpu-baseline --steps 3 --warmup 1 > $GRAFT_REPO_ROOT/gpurun_out/r06o/$v.log 2>&1 || exit 1
done
