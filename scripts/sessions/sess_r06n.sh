# round 6, session n: nd tests with the fronts poisoned (NaN) before the
# solve, prezero off by default; the C5 nd line
bash scripts/gpu_session.sh r06n "tests:tests/test_gpu_solver_nd.py" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline"
