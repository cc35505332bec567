# Selected GPU tests, then library / flag A/Bs on bench workloads.
#   TAG=name TESTS="tests/a.py tests/b.py" VARIANTS="SRF_LIB_PATH=...;..." [WL=wsj_c4]
#   [VARIANTS2="--flag=1;..." WL2=wsj_c5 STEPS2=3] bash scripts/gpu_ab.sh
# Test failures (pytest status 1) do not stop the A/Bs; a crash or a timeout does.
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${TAG:-ab}
rc=0
if [ -n "$TESTS" ]; then
  TAILN=25 TAG=$T bash scripts/gpu_steps.sh \
    "${TLIM:-700}|pytest|python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu $TESTS"
  rc=$?
  [ $rc -gt 1 ] && exit $rc
fi
if [ -n "$VARIANTS" ]; then
  TAG=$T/ab WL=${WL:-wsj_c4} STEPS=${STEPS:-20} VARIANTS="$VARIANTS" bash scripts/gpu_ab_env.sh || exit $?
fi
if [ -n "$VARIANTS2" ]; then
  TAG=$T/ab2 WL=${WL2:-wsj_c5} STEPS=${STEPS2:-3} VTLIM=${VTLIM2:-400} VARIANTS="$VARIANTS2" bash scripts/gpu_ab_env.sh || exit $?
fi
if [ -n "$VARIANTS3" ]; then
  TAG=$T/ab3 WL=${WL3:-wsj_c3} STEPS=${STEPS3:-5} VARIANTS="$VARIANTS3" bash scripts/gpu_ab_env.sh || exit $?
fi
exit $rc
