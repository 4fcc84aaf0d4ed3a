#!/bin/bash
# multi-rank rehearsal on one GPU (gloo carries the all-gather), C2/C3 bench lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
TAG=${1:-r01l}
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/session_$TAG.log
  timeout -k 10 "$t" "$@" > "$OUT/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/session_$TAG.log
  tail -4 "$OUT/${name}_$TAG.log" | tee -a $OUT/session_$TAG.log
  return $rc
}
run dist2_c3 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
    bench.py --gpus 2 --config c3 --steps 3 --warmup 1 --backend gloo --verify || exit $?
run dist3_c2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29512 \
    bench.py --gpus 3 --config c2 --steps 3 --warmup 1 --backend gloo --verify || exit $?
run bench_c3 300 python bench.py --config c3 --steps 20 --warmup 3 || exit $?
run bench_c2 300 python bench.py --config c2 --steps 20 --warmup 3 || exit $?
run verify_c4 600 python bench.py --steps 2 --warmup 1 --no-cpu-baseline --verify
