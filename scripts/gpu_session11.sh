#!/bin/bash
# GPU session: full GPU suite, C4 bench (panelled SpMM), rocprof stats + PMC traffic.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
TAG=${1:-r01k}
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/session_$TAG.log
  timeout -k 10 "$t" "$@" > "$OUT/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/session_$TAG.log
  tail -6 "$OUT/${name}_$TAG.log" | tee -a $OUT/session_$TAG.log
  return $rc
}
run gpu_tests 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider --durations=8 || exit $?
run bench 600 python bench.py || exit $?
export TMPDIR=/tmp
run rocprof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_$TAG -o bench --output-format csv -- \
    python bench.py --steps 5 --warmup 1 --no-cpu-baseline || exit $?
run pmc_fetch 600 rocprofv3 --pmc FETCH_SIZE --kernel-trace -d $OUT/pmc_fetch_$TAG -o pmc --output-format csv -- \
    python bench.py --steps 1 --warmup 0 --no-cpu-baseline || exit $?
run pmc_write 600 rocprofv3 --pmc WRITE_SIZE --kernel-trace -d $OUT/pmc_write_$TAG -o pmc --output-format csv -- \
    python bench.py --steps 1 --warmup 0 --no-cpu-baseline
