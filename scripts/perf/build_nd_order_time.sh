#!/bin/bash
# the host-analysis timer of solve(order="nd") (CPU only); with "ab", also
# the round-5 analysis (scripts/perf/nd_order_r05.cpp) for the same-box A/B
cd "$(dirname "$0")/../.." && mkdir -p scripts/perf/bin && \
g++ -O3 -std=c++20 -pthread -Ibasic_sparse_matrix_amd/csrc scripts/perf/nd_order_time.cpp \
    basic_sparse_matrix_amd/csrc/nd_order.cpp -o scripts/perf/bin/nd_order_time || exit 1
if [ "${1:-}" = ab ]; then
  g++ -O3 -std=c++20 -pthread -Ibasic_sparse_matrix_amd/csrc scripts/perf/nd_order_time.cpp \
      scripts/perf/nd_order_r05.cpp -o scripts/perf/bin/nd_order_time_r05 || exit 1
fi
