#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
TAG=${1:-r01e}
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
run solver_tests 600 python -m pytest tests/test_gpu_solver.py -m gpu -q -p no:cacheprovider -x --durations=8; rc=$?; ok $rc || exit $rc
export TMPDIR=/tmp
run solve_prof 900 rocprofv3 --kernel-trace --stats -d $OUT/prof_solve_$TAG -o solve --output-format csv -- \
    python scripts/solve_c5.py --g 1000 --reps 2; rc=$?
exit $rc
