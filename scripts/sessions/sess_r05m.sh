# round 5, session m: nd factor with pipelined tile loads, corner hints after the band cut
bash scripts/gpu_session.sh r05m \
  "tests:tests/test_gpu_solver_nd.py" \
  "env:BSM_ND_TRACE=1" \
  "py:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 2 --no-cpu-baseline"
