#!/bin/bash
# GPU session: parity tests, SpMM variant A/B at C4, bench, rocprof stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
TAG=${1:-r01b}
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/session_$TAG.log
  timeout -k 10 "$t" "$@" > "$OUT/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/session_$TAG.log
  tail -8 "$OUT/${name}_$TAG.log" | tee -a $OUT/session_$TAG.log
  return $rc
}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
run pytest_gpu 900 python -m pytest tests -m gpu -q -p no:cacheprovider; rc=$?; ok $rc || exit $rc
run variants 900 python scripts/spmm_variants.py; rc=$?; [ $rc -eq 0 ] || exit $rc
run bench 600 python bench.py --steps 5 --warmup 2; rc=$?; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
run rocprof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o bench --output-format csv -- \
    python bench.py --steps 3 --warmup 1 --no-cpu-baseline; rc=$?
exit $rc
