#!/bin/bash
# blocked (reassociated) solve: its tests, the exact solver tests, C5 in both orders under rocprofv3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
TAG=${1:-s41}
timeout -k 10 300 python -u -m pytest tests/test_gpu_solver_blocked.py -x -v -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/blocked_tests_$TAG.log 2>&1 || { tail -40 $OUT/blocked_tests_$TAG.log; exit 1; }
tail -3 $OUT/blocked_tests_$TAG.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c5b_$TAG -o c5 --output-format csv -- python scripts/solve_c5.py --order blocked --reps 3 > $OUT/c5b_prof_$TAG.log 2>&1 || { tail -20 $OUT/c5b_prof_$TAG.log; exit 1; }
grep C5 $OUT/c5b_prof_$TAG.log
