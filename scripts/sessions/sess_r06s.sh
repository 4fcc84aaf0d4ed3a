# round 6, session s: the leaf-level forward and backward solves skip the
# fronts' zero rows and padding columns; nd tests, the C5 nd line, kernel
# stats
bash scripts/gpu_session.sh r06s "tests:tests/test_gpu_solver_nd.py tests/test_gpu_solver.py" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
