#!/bin/bash
# MALL-residency probe: gather rate of the k32 kernel vs X table size
set -o pipefail
mkdir -p gpurun_out
for c in 250000 500000 1000000 2000000 10000000; do
  timeout -k 10 120 python scripts/spmm_variants.py --rows 10000000 --cols $c --nnz-row 50 --variants 3 --rounds 3 \
    >> gpurun_out/mall_probe_r01g.log 2>&1 || exit $?
  echo "cols=$c done" >> gpurun_out/mall_probe_r01g.log
done
timeout -k 10 200 python scripts/spmm_variants.py --rows 2000000 --cols 10000000 --nnz-row 1000 --variants 3 --rounds 3 \
    >> gpurun_out/mall_probe_r01g.log 2>&1
