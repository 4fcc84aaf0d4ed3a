#!/bin/bash
# backward register-window solve: solver parity, then C5 timing + kernel stats
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_solver.py -m gpu -q -x -p no:cacheprovider -k "not c5" > gpurun_out/solver_tests_bw.log 2>&1 || { tail -30 gpurun_out/solver_tests_bw.log; exit 1; }
tail -1 gpurun_out/solver_tests_bw.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5_bw -o c5 --output-format csv -- python scripts/solve_c5.py > gpurun_out/c5_bwprof.log 2>&1 || { tail -20 gpurun_out/c5_bwprof.log; exit 1; }
grep -v amdgpu.ids gpurun_out/c5_bwprof.log | tail -3
python3 -c "
import csv
for r in csv.DictReader(open('gpurun_out/prof_c5_bw/c5_kernel_stats.csv')): print(r['Name'][:70], r['Calls'], float(r['TotalDurationNs'])/1e9)
" | head -5
