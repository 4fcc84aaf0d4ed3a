#!/bin/bash
# Full GPU check: pytest -m gpu (incl. the C++ mirror), smoke(), the default
# bench line, and a C5 solve kernel profile. Usage: scripts/gpu_full.sh TAG
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
TAG=${1:-full}
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/session_$TAG.log
  timeout -k 10 "$t" "$@" > "$OUT/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/session_$TAG.log
  tail -4 "$OUT/${name}_$TAG.log" | tee -a $OUT/session_$TAG.log
  return $rc
}
run gpu_tests 900 python -m pytest tests -m gpu -q -x -p no:cacheprovider --durations=5 || exit $?
run smoke 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" || exit $?
run bench 600 python bench.py || exit $?
export TMPDIR=/tmp
run c5_prof 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_c5_$TAG -o c5 --output-format csv -- \
    python scripts/solve_c5.py
