# wsj_c3 bench step under launch variants (env assignments; 'eager' = --eager), each
# with a kernel trace for scripts/c3_timeline.py:
#   TAG=name VARIANTS="base;DEBUG_HIP_FORCE_GRAPH_QUEUES=8;eager" [NOTRACE=1] [WL=wsj_c4] bash scripts/gpu_c3sched.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-c3sched}
mkdir -p $OUT
B="$GRAFT_REPO_ROOT/bench.py --workload ${WL:-wsj_c3} --extra= --no-cpu-baseline"
cd /tmp && export TMPDIR=/tmp
IFS=';' read -ra VS <<< "${VARIANTS:-base}"
i=0
for v in "${VS[@]}"; do
  i=$((i + 1))
  args=""; envs=""
  for w in $v; do
    case $w in
      base) ;;
      eager) args="$args --eager" ;;
      --*) args="$args $w" ;;
      SRF_LIB_PATH=*) envs="$envs SRF_LIB_PATH=$GRAFT_REPO_ROOT/${w#SRF_LIB_PATH=}" ;;
      *) envs="$envs $w" ;;
    esac
  done
  echo "== [$i] $v"
  echo "== variant [$i]: flags [$args] environment [$envs]" > $OUT/b$i.log
  ( for e in $envs; do export "$e"; done
    timeout -k 10 200 python3 -X faulthandler $B --steps 10 --warmup 3 $args >> $OUT/b$i.log 2>&1 ) || { tail -20 $OUT/b$i.log; exit 1; }
  tail -1 $OUT/b$i.log | python3 -c "import json,sys; d=json.loads(sys.stdin.read()); print('  ms_per_step', d['ms_per_step'])"
  [ -n "$NOTRACE" ] && continue
  ( for e in $envs; do export "$e"; done
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $OUT/kt$i -o run -- \
      python3 $B --steps 4 --warmup 2 $args > $OUT/kt$i.log 2>&1 ) || { tail -20 $OUT/kt$i.log; exit 1; }
  python3 $GRAFT_REPO_ROOT/scripts/c3_timeline.py $OUT/kt$i/run_kernel_trace.csv > $OUT/tl$i.txt
  head -9 $OUT/tl$i.txt
done
echo done
