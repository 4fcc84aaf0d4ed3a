# round 6, session t: the leaf-level forward solve skips the fronts' zero
# rows only (loads unconditional); nd tests, the C5 nd line, kernel stats
bash scripts/gpu_session.sh r06t "tests:tests/test_gpu_solver_nd.py" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
