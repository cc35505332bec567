# C3 (SDR) profile: per-frame recurrence times of the two C3 layer shapes against the
# group size (shipped library, then each library in ABLIBS), the stamp build's phase
# shares, and the kernel-trace statistics of the wsj_c3 bench step.
#   TAG=name [ABLIBS="ab/x.so ..."] bash scripts/gpu_c3prof.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-c3prof}
mkdir -p $OUT
timeout -k 10 150 python3 -u scripts/sdr_group_frames.py > $OUT/groups.log 2>&1 || { tail -5 $OUT/groups.log; exit 1; }
cat $OUT/groups.log
for lib in $ABLIBS; do
  n=$(basename $lib .so)
  SRF_LIB_PATH=$lib timeout -k 10 150 python3 -u scripts/sdr_group_frames.py > $OUT/groups_$n.log 2>&1 || { tail -5 $OUT/groups_$n.log; exit 1; }
  echo "[$lib]"; cat $OUT/groups_$n.log
done
if [ -f ab/stamp.so ]; then
  SRF_LIB_PATH=ab/stamp.so timeout -k 10 150 python3 -u scripts/seq_stamps.py > $OUT/stamps.log 2>&1 || { tail -5 $OUT/stamps.log; exit 1; }
  cat $OUT/stamps.log
fi
B="$GRAFT_REPO_ROOT/bench.py --workload wsj_c3 --extra= --no-cpu-baseline"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt -o run -- \
  python3 $B --steps 5 --warmup 2 > $OUT/kt.log 2>&1 || { tail -20 $OUT/kt.log; exit 1; }
tail -1 $OUT/kt.log
echo done
