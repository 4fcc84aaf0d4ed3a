#!/bin/bash
# band_chol4: parity, trace, and kernel time at C5
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
TAG=${1:-s36}
timeout -k 10 300 python -u -m pytest tests/test_gpu_solver.py -x -q -m gpu --timeout 120 --timeout-method thread -k "cholesky or chol4" -p no:cacheprovider > $OUT/chol_tests_$TAG.log 2>&1 || { tail -20 $OUT/chol_tests_$TAG.log; exit 1; }
tail -1 $OUT/chol_tests_$TAG.log
BSM_CHOL_VARIANT=4 BSM_CHOL_TRACE=1 timeout -k 10 300 python scripts/solve_c5.py > $OUT/c5_trace_$TAG.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/c5_trace_$TAG.log
export TMPDIR=/tmp
BSM_CHOL_VARIANT=4 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c5_chol4_$TAG -o c5 --output-format csv -- python scripts/solve_c5.py > $OUT/c5_chol4_$TAG.log 2>&1 || exit $?
grep C5 $OUT/c5_chol4_$TAG.log
