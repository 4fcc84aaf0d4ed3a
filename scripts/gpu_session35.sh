#!/bin/bash
# C5 kernel times: band_chol4 vs band_chol3 (rocprofv3 kernel trace)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
TAG=${1:-s35}
export TMPDIR=/tmp
BSM_CHOL_VARIANT=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c5_chol4_$TAG -o c5 --output-format csv -- python scripts/solve_c5.py > $OUT/c5_chol4_$TAG.log 2>&1 || exit $?
grep C5 $OUT/c5_chol4_$TAG.log
BSM_CHOL_VARIANT=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c5_chol3_$TAG -o c5 --output-format csv -- python scripts/solve_c5.py > $OUT/c5_chol3_$TAG.log 2>&1 || exit $?
grep C5 $OUT/c5_chol3_$TAG.log
