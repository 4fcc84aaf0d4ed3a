#!/bin/bash
# band_chol3 phase trace at C5
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export BSM_CHOL_TRACE=1
timeout -k 10 300 python scripts/solve_c5.py > gpurun_out/c5_trace_${1:-r01t}.log 2>&1
