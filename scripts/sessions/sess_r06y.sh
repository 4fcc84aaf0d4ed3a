# round 6, session y: the pull's per-task descriptors (BSM_ND_PDESC); nd
# tests, C5 nd pdesc / none / pdesc, the pull's phases
bash scripts/gpu_session.sh r06y "tests:tests/test_gpu_solver_nd.py" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "env:BSM_ND_PDESC=0" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" "unenv:BSM_ND_PDESC" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "env:BSM_ND_STAMPS=1" "py:scripts/solve_c5.py --orders nd --reps 1 --no-cpu-baseline"
