#!/bin/bash
# band_forward2 variants at C5 (wave count x prefetch depth)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
TAG=${1:-r01z}
export TMPDIR=/tmp
for v in 0 2 3 1; do
  BSM_FW_VARIANT=$v timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fw${v}_$TAG -o c5 --output-format csv -- python scripts/solve_c5.py > gpurun_out/c5_fw${v}_$TAG.log 2>&1 || exit 1
  echo "variant $v: $(grep C5 gpurun_out/c5_fw${v}_$TAG.log)"
done
