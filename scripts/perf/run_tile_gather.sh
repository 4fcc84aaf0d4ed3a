#!/bin/bash
# tile_gather sweep (see tile_gather.hip); output to gpurun_out/tile_gather.log
cd "${GRAFT_REPO_ROOT:-.}"
B=scripts/perf/tile_gather
O=gpurun_out/tile_gather.log
mkdir -p gpurun_out
run() { timeout -k 5 60 $B "$@" >> $O 2>&1 || { echo "FAIL $*" >> $O; exit 1; }; }
run 144 8192 1000 1 2
run 144 8192 1000 4 2
XFILL=1 run 144 8192 1000 1 2
XFILL=1 run 144 8192 1000 4 2
echo done >> $O
