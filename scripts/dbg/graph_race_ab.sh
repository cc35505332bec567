# The captured step's gradient race check (scripts/dbg/graph_race.py), two processes
# sharing the GPU.   TAG=name bash scripts/dbg/graph_race_ab.sh [FIXTURE [FLAGS]]
O=gpurun_out/${TAG:-graph_race}
mkdir -p $O
F=${1:-dp2_c2_mini}
(timeout -k 10 200 python -u scripts/dbg/graph_race.py $F 150 $2 > $O/a.log 2>&1 &
 timeout -k 10 200 python -u scripts/dbg/graph_race.py $F 150 $2 > $O/b.log 2>&1; wait)
grep -h SUMMARY $O/a.log $O/b.log
