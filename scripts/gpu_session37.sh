#!/bin/bash
# forward solve (Markstein division, unrolled block, raised priority): solver parity + C5 trace + kernel times
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
TAG=${1:-s37}
timeout -k 10 400 python -u -m pytest tests/test_gpu_solver.py tests/test_gpu_configs.py -x -q -m gpu --timeout 200 --timeout-method thread -p no:cacheprovider > $OUT/solver_tests_$TAG.log 2>&1 || { tail -30 $OUT/solver_tests_$TAG.log; exit 1; }
tail -1 $OUT/solver_tests_$TAG.log
BSM_FW_TRACE=1 timeout -k 10 300 python scripts/solve_c5.py > $OUT/c5_fwtrace_$TAG.log 2>&1 || exit $?
grep -v amdgpu.ids $OUT/c5_fwtrace_$TAG.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c5_$TAG -o c5 --output-format csv -- python scripts/solve_c5.py > $OUT/c5_prof_$TAG.log 2>&1 || exit $?
grep C5 $OUT/c5_prof_$TAG.log
