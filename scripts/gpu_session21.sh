#!/bin/bash
# band_forward2: solver tests + C5 kernel profile
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r01x}
timeout -k 10 300 python -m pytest tests/test_gpu_solver.py -m gpu -q -x -p no:cacheprovider -k "not c5" > gpurun_out/solver_tests_$TAG.log 2>&1 || { tail -30 gpurun_out/solver_tests_$TAG.log; exit 1; }
tail -2 gpurun_out/solver_tests_$TAG.log
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5_$TAG -o c5 --output-format csv -- python scripts/solve_c5.py > gpurun_out/c5_$TAG.log 2>&1 || exit 1
grep C5 gpurun_out/c5_$TAG.log
