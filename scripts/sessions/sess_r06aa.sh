# round 6, session aa: the cold path with the inverse tiles and the flags
# also allocated on the helper thread; after the bench (which frees ~250 GB),
# as in the driver's order; nd tests first
bash scripts/gpu_session.sh r06aa "tests:tests/test_gpu_solver_nd.py" "py:bench.py --steps 2 --warmup 1" \
  "py:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline" \
  "py:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
