#!/bin/bash
# band_chol3 (16 waves, 4-column batches): solver tests + C5 phase trace + C5 timing
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r01u}
timeout -k 10 300 python -m pytest tests/test_gpu_solver.py -m gpu -q -x -p no:cacheprovider -k "not c5" > gpurun_out/solver_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/solver_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/solver_tests_$TAG.log
BSM_CHOL_TRACE=1 timeout -k 10 300 python scripts/solve_c5.py > gpurun_out/c5_trace_$TAG.log 2>&1 || exit 1
grep -v amdgpu.ids gpurun_out/c5_trace_$TAG.log
timeout -k 10 300 python scripts/solve_c5.py > gpurun_out/c5_$TAG.log 2>&1
grep -v amdgpu.ids gpurun_out/c5_$TAG.log
