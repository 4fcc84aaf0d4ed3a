#!/bin/bash
# A/B of the single-pass scan (+ fused k = 1 compaction) against the
# three-launch scan (BSM_SCAN=3) on the C2 / C3 bench steps.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
mkdir -p gpurun_out
for cfg in ${CONFIGS:-c2 c3}; do
  for sc in 1 3; do
    echo "=== $cfg BSM_SCAN=$sc"
    BSM_SCAN=$sc timeout -k 10 180 python bench.py --config $cfg --steps 20 --warmup 3 --no-cpu-baseline --no-e2e \
        > gpurun_out/scan_ab_${cfg}_$sc.log 2>&1 || { echo "rc=$?"; tail -5 gpurun_out/scan_ab_${cfg}_$sc.log; exit 1; }
    grep '^{' gpurun_out/scan_ab_${cfg}_$sc.log | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('ms_per_step', d['ms_per_step'], d['breakdown_ms'])"
  done
done
