# round 5, session an: nd_forward at <= 128 VGPRs (the row terms in two halves): nd tests, C5 timing and kernel trace
bash scripts/gpu_session.sh r05an \
  "tests:tests/test_gpu_solver_nd.py" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
