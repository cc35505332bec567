# Round-4 check: selected GPU tests, then a library A/B on the C4 bench.
#   TAG=name TESTS="tests/a.py tests/b.py" VARIANTS="SRF_LIB_PATH=...;..." bash scripts/gpu_r04.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
T=${TAG:-r04}
TAILN=25 TAG=$T bash scripts/gpu_steps.sh \
  "${TLIM:-700}|pytest|python -u -m pytest -v --timeout 300 --timeout-method thread -m gpu ${TESTS:-tests/}" || exit $?
if [ -n "$VARIANTS" ]; then
  TAG=$T/ab WL=${WL:-wsj_c4} STEPS=${STEPS:-20} VARIANTS="$VARIANTS" bash scripts/gpu_ab_env.sh
fi
