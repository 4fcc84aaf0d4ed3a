# round 6, session q: the host analysis with the bisection's block pool
# against the build before it (scripts/perf/nd_order_prev.cpp: the previous
# commit's nd_order.cpp), alternating, on the box's CPUs
# (To rerun: the A/B side is not committed; recreate scripts/perf/nd_order_prev.cpp
# first with git show <commit before the session>:basic_sparse_matrix_amd/csrc/nd_order.cpp.)
bash scripts/perf/build_nd_order_time.sh && \
g++ -O3 -std=c++20 -pthread -Ibasic_sparse_matrix_amd/csrc scripts/perf/nd_order_time.cpp \
    scripts/perf/nd_order_prev.cpp -o scripts/perf/bin/nd_order_time_prev && \
bash scripts/gpu_session.sh r06q \
  "cmd:scripts/perf/bin/nd_order_time_prev 1000 192 16" "cmd:scripts/perf/bin/nd_order_time 1000 192 16" \
  "cmd:scripts/perf/bin/nd_order_time_prev 1000 192 16" "cmd:scripts/perf/bin/nd_order_time 1000 192 16" \
  "cmd:scripts/perf/bin/nd_order_time_prev 1000 192 16" "cmd:scripts/perf/bin/nd_order_time 1000 192 16"
