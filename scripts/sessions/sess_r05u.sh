# round 5, session u: nd field cuts on records, device BFS with one barrier per level
T=scripts/perf/bin/nd_order_time
bash scripts/gpu_session.sh r05u \
  "tests:tests/test_gpu_solver_nd.py" \
  "env:BSM_ND_TRACE=2" "cmd:$T 1000 192 16" \
  "py:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline" \
  "env:BSM_ND_FIELDS=0" "py:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
