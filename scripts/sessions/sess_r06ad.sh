# round 6, session ad: the leaf-level backward solve reads a real row's
# address for L's zero rows; nd tests, the C5 nd line, kernel stats
bash scripts/gpu_session.sh r06ad "tests:tests/test_gpu_solver_nd.py tests/test_gpu_solver.py" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
