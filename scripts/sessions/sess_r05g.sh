# round 5, session g: the nested-dissection solve (order="nd") -- GPU tests, then C5 timings of all orders
bash scripts/gpu_session.sh r05g \
  "tests:tests/test_gpu_solver_nd.py" \
  "tests:tests/test_gpu_solver_blocked.py" \
  "env:BSM_ND_TRACE=1" \
  "py:scripts/solve_c5.py --orders nd,blocked --reps 2 --no-cpu-baseline"
