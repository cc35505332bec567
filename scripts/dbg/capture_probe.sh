set -o pipefail
cd $GRAFT_REPO_ROOT
for w in torch stackfwd step; do
  timeout -k 10 120 python -u scripts/dbg/capture_probe.py $w > gpurun_out/probe_$w.log 2>&1
  rc=$?
  echo "$w rc=$rc"; tail -3 gpurun_out/probe_$w.log
  [ $rc -ne 0 ] && exit $rc
done
exit 0
