#!/bin/bash
# SpMV v2 (batched loads): tests, chunk A/B at C2, C2 bench
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
TAG=${1:-r01n}
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
run spmv_c2 300 python scripts/spmm_variants.py --rows 1000000 --cols 1000000 --nnz-row 10 --k 1 --env BSM_SPMV_ITEMS --variants 4,2,8 --rounds 10 || exit $?
run spmv_big 300 python scripts/spmm_variants.py --rows 20000000 --cols 20000000 --nnz-row 10 --k 1 --env BSM_SPMV_ITEMS --variants 4,2,8 --rounds 5 || exit $?
run bench_c2 300 python bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline
