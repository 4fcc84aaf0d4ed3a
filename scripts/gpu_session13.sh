#!/bin/bash
# short-row k32 kernel + wave search SpMV: tests, A/B at C3, C2/C3 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
TAG=${1:-r01m}
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/session_$TAG.log
  timeout -k 10 "$t" "$@" > "$OUT/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/session_$TAG.log
  tail -7 "$OUT/${name}_$TAG.log" | tee -a $OUT/session_$TAG.log
  return $rc
}
run spmm_tests 600 python -m pytest tests/test_gpu_spmm.py tests/test_gpu_configs.py -m gpu -q -x -p no:cacheprovider || exit $?
run variants_c3 300 python scripts/spmm_variants.py --rows 1000000 --cols 1000000 --nnz-row 10 --variants 3,5,6,1 --rounds 5 || exit $?
run variants_24 300 python scripts/spmm_variants.py --rows 1000000 --cols 1000000 --nnz-row 24 --variants 3,5,6 --rounds 5 || exit $?
run variants_48 300 python scripts/spmm_variants.py --rows 1000000 --cols 1000000 --nnz-row 48 --variants 3,5 --rounds 5 || exit $?
run bench_c3 300 python bench.py --config c3 --steps 20 --warmup 3 --no-cpu-baseline || exit $?
run bench_c2 300 python bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline
