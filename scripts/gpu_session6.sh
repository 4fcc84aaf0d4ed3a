#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
TAG=${1:-r01f}
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/session_$TAG.log
  timeout -k 10 "$t" "$@" > "$OUT/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/session_$TAG.log
  tail -15 "$OUT/${name}_$TAG.log" | tee -a $OUT/session_$TAG.log
  return $rc
}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
run solver_tests 600 python -m pytest tests/test_gpu_solver.py -m gpu -q -p no:cacheprovider --durations=8; rc=$?; ok $rc || exit $rc
BSM_CHOL_TRACE=1 run solve_trace 600 python scripts/solve_c5.py --g 1000 --reps 1; rc=$?; [ $rc -eq 0 ] || exit $rc
BSM_CHOL_TRACE=1 run solve_trace250 600 python scripts/solve_c5.py --g 250 --reps 1; rc=$?
exit $rc
