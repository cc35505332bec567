# Stream ring depth A/B after the run-ahead fix: C5 fp32 and fp8, default vs ab/pdb, ab/pdc.
set -o pipefail
cd $GRAFT_REPO_ROOT
LIBS="ab/pdb.so ab/pdc.so" TAG=r04ff/c5 timeout -k 10 700 bash scripts/gpu_lib_ab_c5.sh || exit $?
WL=wsj_c5_fp8 LIBS="ab/pdb.so ab/pdc.so" TAG=r04ff/c5fp8 timeout -k 10 700 bash scripts/gpu_lib_ab_c5.sh
