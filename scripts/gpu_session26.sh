#!/bin/bash
# backward register-window variants: solver parity, C5 per variant, kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_solver.py -m gpu -q -x -p no:cacheprovider -k "not c5" > gpurun_out/solver_tests_bw.log 2>&1 || { tail -30 gpurun_out/solver_tests_bw.log; exit 1; }
tail -1 gpurun_out/solver_tests_bw.log
export TMPDIR=/tmp
for v in 0 5 4; do
  BSM_BW_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5_bw$v -o c5 --output-format csv -- python scripts/solve_c5.py > gpurun_out/c5_bwprof$v.log 2>&1 || { tail -20 gpurun_out/c5_bwprof$v.log; exit 1; }
  echo "variant $v: $(grep 'solve wall' gpurun_out/c5_bwprof$v.log)"
  python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_c5_bw$v/c5_kernel_stats.csv')):
    if 'band_' in r['Name']: print('  ', r['Name'][:75], float(r['TotalDurationNs'])/1e9)
"
done
