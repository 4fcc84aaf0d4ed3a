#!/bin/bash
# the host-analysis timer of solve(order="nd") (CPU only)
cd "$(dirname "$0")/../.." && mkdir -p scripts/perf/bin && \
g++ -O3 -std=c++20 -pthread -Ibasic_sparse_matrix_amd/csrc scripts/perf/nd_order_time.cpp \
    basic_sparse_matrix_amd/csrc/nd_order.cpp -o scripts/perf/bin/nd_order_time
