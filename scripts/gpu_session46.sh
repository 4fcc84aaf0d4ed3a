#!/bin/bash
# blocked Cholesky: tests, a traced C5 run (BSM_BLK_DEBUG: per-phase cycles), C5 under rocprofv3
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
TAG=${1:-s46}
export BSM_BLK_WATCH=1
timeout -k 10 300 python -u -m pytest tests/test_gpu_solver_blocked.py -x -q -m gpu --timeout 120 --timeout-method thread -p no:cacheprovider > $OUT/blocked_tests_$TAG.log 2>&1 || { tail -30 $OUT/blocked_tests_$TAG.log; exit 1; }
tail -1 $OUT/blocked_tests_$TAG.log
BSM_BLK_DEBUG=1 timeout -k 10 120 python -u scripts/solve_c5.py --order blocked > $OUT/c5b_trace_$TAG.log 2>&1 || { tail -5 $OUT/c5b_trace_$TAG.log; exit 1; }
grep -E "blk debug|C5" $OUT/c5b_trace_$TAG.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $OUT/prof_c5b_$TAG -o c5 --output-format csv -- python scripts/solve_c5.py --order blocked --reps 2 > $OUT/c5b_prof_$TAG.log 2>&1 || { tail -20 $OUT/c5b_prof_$TAG.log; exit 1; }
grep C5 $OUT/c5b_prof_$TAG.log
python3 - <<PY
import csv
for r in csv.DictReader(open('$OUT/prof_c5b_$TAG/c5_kernel_stats.csv')):
    if float(r['AverageNs']) > 1e6: print(r['Name'][:50], r['Calls'], round(float(r['AverageNs'])/1e6, 2), 'ms')
PY
