#!/bin/bash
# column-panel SpMM: parity tests, then width A/B at C4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_spmm.py tests/test_gpu_configs.py -x -q -m gpu \
   > gpurun_out/spmm_tests_r01h.log 2>&1 || exit $?
timeout -k 10 400 python scripts/spmm_panels.py --widths 0,2000000,1000000,500000,250000 \
   > gpurun_out/spmm_panels_r01h.log 2>&1
