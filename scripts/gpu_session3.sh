#!/bin/bash
# GPU session: solver tests first (new kernels), full GPU suite, PMC traffic of the SpMM kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
TAG=${1:-r01c}
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
run solver_small 300 python -m pytest tests/test_gpu_solver.py -m gpu -q -x -p no:cacheprovider -k "not 250 and not c5" --durations=10; rc=$?; ok $rc || exit $rc
run solver_big 600 python -m pytest tests/test_gpu_solver.py -m gpu -q -p no:cacheprovider -k "250 or c5" --durations=5; rc=$?; ok $rc || exit $rc
export TMPDIR=/tmp
run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch_$TAG -o pmc --output-format csv -- \
    python scripts/spmm_variants.py --variants 3 --rounds 1; rc=$?; [ $rc -eq 0 ] || exit $rc
run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write_$TAG -o pmc --output-format csv -- \
    python scripts/spmm_variants.py --variants 3 --rounds 1; rc=$?
exit $rc
