#!/bin/bash
# backward chain segment length A/B at C5 (SEG 32 default vs 16), solver tests
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
TAG=${1:-r01q}
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/session_$TAG.log
  timeout -k 10 "$t" "$@" > "$OUT/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/session_$TAG.log
  tail -4 "$OUT/${name}_$TAG.log" | tee -a $OUT/session_$TAG.log
  return $rc
}
run solver_tests 900 python -m pytest tests/test_gpu_solver.py -m gpu -q -x -p no:cacheprovider -k "not c5" || exit $?
export TMPDIR=/tmp
run c5_seg32 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_c5_$TAG -o c5 --output-format csv -- \
    python scripts/solve_c5.py || exit $?
export BSM_BW_VARIANT=2
run c5_seg16 600 python scripts/solve_c5.py
