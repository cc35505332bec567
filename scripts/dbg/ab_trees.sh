# C4 step time of two source trees on one box, alternating: the repo and ab/old.
#   TAG=name bash scripts/dbg/ab_trees.sh
O=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-abtrees}
mkdir -p $O
for k in 1 2 3; do
  for t in new old; do
    d=$GRAFT_REPO_ROOT; [ $t = old ] && d=$GRAFT_REPO_ROOT/ab/old
    (cd $d && timeout -k 10 300 python -u bench.py --workload wsj_c4 --extra= --no-cpu-baseline --steps 20 --warmup 3 \
      > $O/$t$k.json 2> $O/$t$k.err) || { echo "$t$k failed"; tail -3 $O/$t$k.err; exit 1; }
    python -c "import json; d=json.load(open('$O/$t$k.json')); print('$t', d['ms_per_step'])"
  done
done
