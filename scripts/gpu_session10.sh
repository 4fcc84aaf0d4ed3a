#!/bin/bash
# kernel ceiling: gather rate with L2/MALL-resident X tables
set -o pipefail
mkdir -p gpurun_out
for c in 16000 100000 1000000; do
  timeout -k 10 120 python scripts/spmm_variants.py --rows 2000000 --cols $c --nnz-row 1000 --variants 3,4,2 --rounds 3 \
    >> gpurun_out/kernel_ceiling_r01j.log 2>&1 || exit $?
  echo "cols=$c done" >> gpurun_out/kernel_ceiling_r01j.log
done
