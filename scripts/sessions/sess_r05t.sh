# round 5, session t: nd bisection by distance fields (device BFS), tests and C5 cold/warm
bash scripts/gpu_session.sh r05t \
  "tests:tests/test_gpu_solver_nd.py" \
  "env:BSM_ND_TRACE=1" \
  "py:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
