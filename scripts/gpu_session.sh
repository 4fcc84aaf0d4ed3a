#!/bin/bash
# One gpurun session: GPU parity tests, a short bench, a rocprofv3 kernel
# trace of the bench. Every GPU step has its own time limit; the script stops
# at the first crash / timeout (exit >= 124 or signal) and only continues past
# ordinary test failures (pytest exit 1).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
TAG=${1:-r01}
run() {  # name timeout cmd...
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/session_$TAG.log
  timeout -k 10 "$t" "$@" > "$OUT/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/session_$TAG.log
  tail -5 "$OUT/${name}_$TAG.log" | tee -a $OUT/session_$TAG.log
  return $rc
}
ok() { [ "$1" -eq 0 ] || [ "$1" -eq 1 ]; }
rocm-smi --showproductname > $OUT/smi_$TAG.log 2>&1 || true
run pytest_gpu 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider; rc=$?; ok $rc || exit $rc
run bench 600 python bench.py --steps 5 --warmup 2; rc=$?; [ $rc -eq 0 ] || exit $rc
export TMPDIR=/tmp
run rocprof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o bench --output-format csv -- \
    python bench.py --steps 3 --warmup 1 --no-cpu-baseline; rc=$?
exit $rc
