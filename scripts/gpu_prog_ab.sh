set -e
cd $GRAFT_REPO_ROOT
OUT=gpurun_out/r02_prog; mkdir -p $OUT
for v in dbg4 progdbg4; do SRF_LIB_PATH=$PWD/ab/$v.so timeout -k 10 120 python scripts/bench_route.py --layers 3 --iters 3 > $OUT/$v.txt 2>&1; grep "blk 100" $OUT/$v.txt | tail -4; done
TAG=r02_prog ALT="prog early" ROUTE=1,3 bash scripts/gpu_libab.sh
