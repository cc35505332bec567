# Race check (scripts/dbg/graph_race.py, two processes) and C4 step time, default
# (one stream) against the side-stream launches (ops.DR_GW_SIDE / CNNFE_WGRAD_SIDE).
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-raceperf}
mkdir -p $O
for v in "" "--side"; do
  n=x$v
  (timeout -k 10 240 python -u scripts/dbg/graph_race.py dp2_c2_mini 300 $v > $O/$n.a.log 2>&1 &
   timeout -k 10 240 python -u scripts/dbg/graph_race.py dp2_c2_mini 300 $v > $O/$n.b.log 2>&1; wait)
  echo "[$v]"; grep -h SUMMARY $O/$n.a.log $O/$n.b.log || exit 1
done
for k in 1 2 3; do
  for v in "" "--side-streams"; do
    timeout -k 10 300 python -u bench.py --workload wsj_c4 --extra= --no-cpu-baseline --steps 20 --warmup 3 $v \
      > $O/b$k.json 2> $O/b$k.err || { tail -3 $O/b$k.err; exit 1; }
    python -c "import json; d=json.load(open('$O/b$k.json')); print('[$v]', d['ms_per_step'])"
  done
done
