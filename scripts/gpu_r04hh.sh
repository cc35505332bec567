# C5 fp8 A/B of the backward ring depth with bf16 u: default (4, 2) vs ab/bb (6, 3), ab/bc (8, 4).
set -o pipefail
cd $GRAFT_REPO_ROOT
WL=wsj_c5_fp8 LIBS="ab/bb.so ab/bc.so" TAG=r04hh/c5fp8 timeout -k 10 700 bash scripts/gpu_lib_ab_c5.sh
