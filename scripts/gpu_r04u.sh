# DR gW on a second stream during the training backward: model / train / DP tests, then
# a C4 A/B against the single-stream backward.
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=r04u TAILN=6 bash scripts/gpu_steps.sh \
  "400|pytest|python -u -m pytest -q --timeout 300 --timeout-method thread -m gpu tests/test_model_gpu.py tests/test_train_gpu.py tests/test_dp_gpu.py tests/test_parity_scale_gpu.py"
rc=$?
[ $rc -gt 1 ] && exit $rc
TAG=r04u/ab WL=wsj_c4 STEPS=20 VARIANTS="--dr-gw-main-stream;SRF_X=1;--dr-gw-main-stream;SRF_X=1;--dr-gw-main-stream;SRF_X=1" bash scripts/gpu_ab_env.sh || exit $?
exit $rc
