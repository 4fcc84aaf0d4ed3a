# round 5, session ab: nd numeric buffers kept on the cached plan; diagonal tiles skip their padding panels
bash scripts/gpu_session.sh r05ab \
  "tests:tests/test_gpu_solver_nd.py" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "env:BSM_ND_PAD_SKIP=0" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "unenv:BSM_ND_PAD_SKIP" \
  "env:BSM_ND_KEEP=0" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "unenv:BSM_ND_KEEP" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
