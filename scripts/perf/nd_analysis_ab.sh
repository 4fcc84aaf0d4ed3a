#!/bin/bash
# same-box A/B of the nd host analysis at C5 (g = 1000, leaf 192): the
# round-5 analysis against HEAD's, 16 threads (the library's default on a
# 16-CPU share), five runs each, alternating
cd "$(dirname "$0")/../.." && bash scripts/perf/build_nd_order_time.sh ab || exit 1
for i in 1 2 3 4 5; do
  echo -n "r05  "; ./scripts/perf/bin/nd_order_time_r05 1000 192 16 | tail -1
  echo -n "head "; ./scripts/perf/bin/nd_order_time 1000 192 16 | tail -1
done
