#!/bin/bash
# The L2-served gather ceiling of the tiled SpMM's inner loop (tile_gather.hip:
# the same six-phase pipeline, 16-B/lane gathers of 256-B X rows, LDS
# read-add-write of 64 distinct rows per chunk), by X table size. COLMASK
# folds every column into the first COLMASK+1 X rows: 8191 = a static 2 MiB
# table that stays in every XCD's 4 MiB L2. bench.py's roofline_gather peak is
# the "mode 2, 2 MiB" line. Output: gpurun_out/gather_ceiling.log
cd "${GRAFT_REPO_ROOT:-.}"
B=scripts/perf/tile_gather
O=gpurun_out/gather_ceiling.log
mkdir -p gpurun_out
: > $O
run() { echo "# $*" >> $O; timeout -k 5 60 $B "$@" >> $O 2>&1 || { echo "FAIL $*" >> $O; exit 1; }; }
# RW PANEL_COLS N_PANELS BATCHES MODE COLMASK
run 155 4096 1000 1 2 8191      # static 2 MiB table, LDS update (the kernel's inner loop)
run 155 4096 1000 1 1 8191      # static 2 MiB table, register sums only (gathers alone)
run 155 4096 1000 1 2 65535     # 16 MiB: spills the L2, Infinity Cache
run 155 4096 1000 1 2 1048575   # 256 MiB: the Infinity Cache's size
run 155 4096 1000 1 2           # the real panel sweep over 10M columns (C4-like stream)
echo done >> $O
