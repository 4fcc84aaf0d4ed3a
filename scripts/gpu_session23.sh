#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for v in 0 3; do
  BSM_FW_TRACE=1 BSM_FW_VARIANT=$v timeout -k 10 300 python scripts/solve_c5.py > gpurun_out/c5_fwtrace${v}.log 2>&1 || exit 1
  echo "variant $v:"; grep -v amdgpu.ids gpurun_out/c5_fwtrace${v}.log
done
