#!/bin/bash
# GPU session: scripts/gpu_session.sh TAG STEP...
# STEP: tests | tests:<paths> | smoke | bench:<config>[:extra bench args] | prof:<config>[:extra]
#       | pmc:<config>:<COUNTER[,COUNTER...]>[:extra] | c5 | gather | torchrun:<config>[:extra]
#       | py:<script args> | profpy:<name>:<script args> (the script under rocprofv3 --kernel-trace --stats)
#       | cmd:<program args> (a built binary, e.g. a probe) | env:VAR=VALUE (for the later steps) | unenv:VAR
# Every step runs under its own time limit; the session stops at the first
# failing step (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
OUT=gpurun_out
TAG=$1
shift
export TMPDIR=/tmp
run() {
  local name=$1 t=$2; shift 2
  echo "=== $name: $*" | tee -a $OUT/session_$TAG.log
  timeout -k 10 "$t" "$@" > "$OUT/${name}_$TAG.log" 2>&1
  local rc=$?
  echo "=== $name rc=$rc" | tee -a $OUT/session_$TAG.log
  tail -3 "$OUT/${name}_$TAG.log" | cut -c1-600 | tee -a $OUT/session_$TAG.log
  return $rc
}
n=0
for step in "$@"; do
  case $step in
    tests) run gpu_tests 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 150 \
             --timeout-method thread --durations=8 || exit $? ;;
    tests:*) n=$((n + 1)); run gpu_tests_sel${n} 600 python -u -m pytest ${step#tests:} -m gpu -x -q -p no:cacheprovider \
             --timeout 150 --timeout-method thread --durations=8 || exit $? ;;
    smoke) run smoke 300 python -c "import __graft_entry__ as g; g.smoke()" || exit $? ;;
    bench:*) IFS=: read -r _ cfg extra <<< "$step"
             run bench_$cfg 600 python bench.py --config $cfg $extra || exit $? ;;
    prof:*) IFS=: read -r _ cfg extra <<< "$step"
            run prof_$cfg 600 rocprofv3 --kernel-trace --stats -d $OUT/prof_${cfg}_$TAG -o run \
                --output-format csv -- python bench.py --config $cfg --no-cpu-baseline --no-e2e $extra || exit $? ;;
    pmc:*) IFS=: read -r _ cfg ctr extra <<< "$step"  # counters joined by ',' (one pass)
           cn=${ctr//,/_}
           [ -n "$extra" ] && cn="${cn}_$(echo "$extra" | tr -c 'a-zA-Z0-9' '_' | cut -c1-40)"
           run pmc_${cfg}_${cn} 300 rocprofv3 --pmc ${ctr//,/ } -d $OUT/pmc_${cfg}_${cn}_$TAG -o run \
               --output-format csv -- python bench.py --config $cfg --steps 2 --warmup 0 --no-cpu-baseline \
               --no-e2e $extra || exit $? ;;
    gather) run gather 300 bash scripts/perf/gather_ceiling.sh || exit $? ;;
    torchrun:*) IFS=: read -r _ cfg extra <<< "$step"
                run torchrun_$cfg 600 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 \
                    --master-addr 127.0.0.1 --master-port 29533 bench.py --gpus 1 --config $cfg $extra || exit $? ;;
    c5) run c5 600 python scripts/solve_c5.py || exit $? ;;
    py:*) n=$((n + 1)); run py${n} 600 python ${step#py:} || exit $? ;;
    cmd:*) n=$((n + 1)); run cmd${n} 300 ${step#cmd:} || exit $? ;;
    profpy:*) IFS=: read -r _ nm args <<< "$step"
              run profpy_$nm 600 rocprofv3 --kernel-trace --stats -d $OUT/profpy_${nm}_$TAG -o run \
                  --output-format csv -- python $args || exit $? ;;
    env:*) export "${step#env:}"; echo "=== export ${step#env:}" | tee -a $OUT/session_$TAG.log ;;
    unenv:*) unset "${step#unenv:}" ;;
    *) echo "unknown step $step"; exit 2 ;;
  esac
done
echo "=== session $TAG done" | tee -a $OUT/session_$TAG.log
