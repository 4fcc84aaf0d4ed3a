#!/bin/bash
# block-cyclic overlapped all-gather: N=1 chunk cost and multi-rank rehearsal (gloo, ranks share the GPU)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
TAG=${1:-s27}
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/session_$TAG.log
  timeout -k 10 "$t" "$@" > "$OUT/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/session_$TAG.log
  tail -3 "$OUT/${name}_$TAG.log" | tee -a $OUT/session_$TAG.log
  return $rc
}
run c4_chunks1 300 python bench.py --no-cpu-baseline --chunks 1 || exit $?
run c4_chunks4 300 python bench.py --no-cpu-baseline --chunks 4 || exit $?
run dist2_c3 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 --master-port 29511 \
    bench.py --gpus 2 --config c3 --steps 3 --warmup 1 --backend gloo --verify || exit $?
run dist3_c2 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 3 --master-addr 127.0.0.1 --master-port 29512 \
    bench.py --gpus 3 --config c2 --steps 3 --warmup 1 --backend gloo --verify --chunks 3 || exit $?
