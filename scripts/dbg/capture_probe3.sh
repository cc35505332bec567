cd $GRAFT_REPO_ROOT
timeout -k 10 120 python -u scripts/dbg/capture_probe2.py torch2fork > gpurun_out/probe3a.log 2>&1
echo "torch2fork rc=$?"; grep -v amdgpu.ids gpurun_out/probe3a.log | tail -2
timeout -k 10 120 python -u scripts/dbg/capture_probe2.py step > gpurun_out/probe3.log 2>&1
echo "step rc=$?"; grep -v amdgpu.ids gpurun_out/probe3.log | tail -2
exit 0
