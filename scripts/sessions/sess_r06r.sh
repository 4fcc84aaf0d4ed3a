# round 6, session r: the host analysis with the child graphs extracted on
# several threads at the top depths, against the build before it
# (scripts/perf/nd_order_prev.cpp: the previous commit's nd_order.cpp),
# alternating, on the box's CPUs. To rerun: the A/B side is not committed;
# recreate it first, e.g. git show 8f24793~1:basic_sparse_matrix_amd/csrc/nd_order.cpp
# > scripts/perf/nd_order_prev.cpp (and the tested side from the session's
# working tree); then the C5 nd line
# (To rerun: the A/B side is not committed; recreate scripts/perf/nd_order_prev.cpp
# first with git show <commit before the session>:basic_sparse_matrix_amd/csrc/nd_order.cpp.)
bash scripts/perf/build_nd_order_time.sh && \
g++ -O3 -std=c++20 -pthread -Ibasic_sparse_matrix_amd/csrc scripts/perf/nd_order_time.cpp \
    scripts/perf/nd_order_prev.cpp -o scripts/perf/bin/nd_order_time_prev && \
bash scripts/gpu_session.sh r06r "env:BSM_ND_TRACE=2" \
  "cmd:scripts/perf/bin/nd_order_time_prev 1000 192 16" "cmd:scripts/perf/bin/nd_order_time 1000 192 16" \
  "cmd:scripts/perf/bin/nd_order_time_prev 1000 192 16" "cmd:scripts/perf/bin/nd_order_time 1000 192 16" \
  "cmd:scripts/perf/bin/nd_order_time_prev 1000 192 16" "cmd:scripts/perf/bin/nd_order_time 1000 192 16" \
  "unenv:BSM_ND_TRACE" "py:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
