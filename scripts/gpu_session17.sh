#!/bin/bash
# band_chol3: solver tests (both Cholesky kernels), C5 timing + trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
TAG=${1:-r01s}
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/session_$TAG.log
  timeout -k 10 "$t" "$@" > "$OUT/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/session_$TAG.log
  tail -6 "$OUT/${name}_$TAG.log" | tee -a $OUT/session_$TAG.log
  return $rc
}
run solver_small 300 python -m pytest tests/test_gpu_solver.py -m gpu -q -x -p no:cacheprovider -k "not c5 and not 250" || exit $?
run solver_250 300 python -m pytest tests/test_gpu_solver.py -m gpu -q -x -p no:cacheprovider -k "250" || exit $?
export TMPDIR=/tmp
export BSM_CHOL_TRACE=1
run c5_chol3 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_c5_$TAG -o c5 --output-format csv -- \
    python scripts/solve_c5.py
