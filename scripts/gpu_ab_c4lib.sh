# C4 bench over (library, env) variants, one process each:
#   TAG=name VARIANTS="SRF_LIB_PATH=ab/x.so A=1;A=0" bash scripts/gpu_ab_c4lib.sh
set -o pipefail
cd $GRAFT_REPO_ROOT
TAG=${TAG:-c4lib} WL=${WL:-wsj_c4} STEPS=${STEPS:-20} bash scripts/gpu_ab_env.sh
