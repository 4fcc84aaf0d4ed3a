#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python -m pytest tests/test_gpu_solver.py -m gpu -q -x -p no:cacheprovider -k "not c5" > gpurun_out/solver_tests_fw.log 2>&1 || { tail -30 gpurun_out/solver_tests_fw.log; exit 1; }
tail -1 gpurun_out/solver_tests_fw.log
for v in 0 3; do
  BSM_FW_TRACE=1 BSM_FW_VARIANT=$v timeout -k 10 300 python scripts/solve_c5.py > gpurun_out/c5_fwtrace${v}.log 2>&1 || exit 1
  echo "variant $v:"; grep -v amdgpu.ids gpurun_out/c5_fwtrace${v}.log
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_c5_fw -o c5 --output-format csv -- python scripts/solve_c5.py > gpurun_out/c5_fwprof.log 2>&1
