#!/bin/bash
# C2 A/B of the k = 1 tiled kernel's load flavours (BSM_TILED_K1_LOADS, see
# kernels_tiled.hip): one bench line per flavour, kernel time from HIP events.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for lm in ${LOADS:-0 1 2 3 4 5 0}; do
  echo "=== BSM_TILED_K1_LOADS=$lm"
  BSM_TILED_K1_LOADS=$lm timeout -k 10 180 python bench.py --config c2 --steps 20 --warmup 3 --no-cpu-baseline \
      --no-e2e > gpurun_out/k1_loads_$lm.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/k1_loads_$lm.log; exit 1; }
  grep '^{' gpurun_out/k1_loads_$lm.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms_per_step', d['ms_per_step'], 'kernel_ms', d['breakdown_ms']['spmm_kernel_mean'], 'frac', d['roofline']['frac'])"
done
