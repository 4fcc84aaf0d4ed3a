# round 5, session n: nd factor, pipelined loads with LDS-only barriers
bash scripts/gpu_session.sh r05n \
  "tests:tests/test_gpu_solver_nd.py" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
