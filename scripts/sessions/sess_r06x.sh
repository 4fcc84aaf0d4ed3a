# round 6, session x: each factor tile stages its own entries of A from the
# plan's per-tile lists (BSM_ND_APULL; no zeroing, no assembly); nd tests,
# C5 nd apull / zero+assemble / apull, kernel stats
bash scripts/gpu_session.sh r06x "tests:tests/test_gpu_solver_nd.py" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "env:BSM_ND_APULL=0" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" "unenv:BSM_ND_APULL" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
