#!/bin/bash
# band_chol4 (tile-event Cholesky): parity tests, then C5 timing vs band_chol3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
TAG=${1:-s28}
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/session_$TAG.log
  timeout -k 10 "$t" "$@" > "$OUT/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/session_$TAG.log
  tail -5 "$OUT/${name}_$TAG.log" | tee -a $OUT/session_$TAG.log
  return $rc
}
run chol_tests 300 python -u -m pytest tests/test_gpu_solver.py -x -v -m gpu --timeout 120 --timeout-method thread -k "cholesky or chol4" -p no:cacheprovider || exit $?
export TMPDIR=/tmp
BSM_CHOL_VARIANT=4 run c5_chol4 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c5_chol4_$TAG -o c5 --output-format csv -- python scripts/solve_c5.py || exit $?
