cd $GRAFT_REPO_ROOT
for w in torchbwd torchbwd_relaxed torchbwd_tl step_relaxed step_tl; do
  timeout -k 10 120 python -u scripts/dbg/capture_probe2.py $w > gpurun_out/probe2_$w.log 2>&1
  rc=$?
  echo "$w rc=$rc"; grep -v amdgpu.ids gpurun_out/probe2_$w.log | tail -2
done
exit 0
