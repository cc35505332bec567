# Runs GPU steps in order, each under its own time limit; stops at the first step
# that crashes, aborts or times out (exit status other than 0 or 1 = test failures).
#   TAG=name bash scripts/gpu_steps.sh 'SECONDS|name|command' ...
# Each step's output goes to gpurun_out/$TAG/<name>.log; its tail is printed.
set -o pipefail
cd $GRAFT_REPO_ROOT
OUT=$GRAFT_REPO_ROOT/gpurun_out/${TAG:-steps}
mkdir -p $OUT
final=0
for spec in "$@"; do
  lim=${spec%%|*}; rest=${spec#*|}; name=${rest%%|*}; cmd=${rest#*|}
  echo "== $name ($lim s): $cmd"
  timeout -k 10 $lim bash -c "$cmd" > $OUT/$name.log 2>&1
  rc=$?
  tail -${TAILN:-12} $OUT/$name.log
  echo "== $name rc=$rc"
  if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then exit $rc; fi
  [ $rc -ne 0 ] && final=$rc
done
exit $final
