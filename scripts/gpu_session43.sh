#!/bin/bash
# blocked Cholesky: a first small test alone (short limit), then the blocked suite and C5
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
TAG=${1:-s43}
timeout -k 10 90 python -u -m pytest "tests/test_gpu_solver_blocked.py::test_blocked_solve_golden" -x -q -m gpu --timeout 40 --timeout-method thread -p no:cacheprovider > $OUT/blocked_first_$TAG.log 2>&1 || { tail -5 $OUT/blocked_first_$TAG.log; exit 1; }
tail -1 $OUT/blocked_first_$TAG.log
bash scripts/gpu_session41.sh $TAG
