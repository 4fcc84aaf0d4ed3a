# round 5, session s: nd bisection on a LIFO worker pool (host timer, then C5 cold/warm and the nd tests)
T=scripts/perf/bin/nd_order_time
bash scripts/gpu_session.sh r05s \
  "cmd:$T 1000 192 16" \
  "env:BSM_ND_TRACE=2" "cmd:$T 1000 192 16" "unenv:BSM_ND_TRACE" \
  "tests:tests/test_gpu_solver_nd.py" \
  "env:BSM_ND_TRACE=1" \
  "py:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
