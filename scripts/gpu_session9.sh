#!/bin/bash
# panel width sweep at C4
set -o pipefail
mkdir -p gpurun_out
timeout -k 10 500 python scripts/spmm_panels.py --widths 0,5000000,3333334,2500000,2000000,1500000 \
   > gpurun_out/spmm_panels_r01i.log 2>&1
