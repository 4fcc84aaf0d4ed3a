# round 6, session k: the pull with the tile staged by coalesced columns,
# unconditional clamped loads and read-then-write additions; nd tests, C5 nd
# (pull, push), the pull's phases
bash scripts/gpu_session.sh r06k "tests:tests/test_gpu_solver_nd.py" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "env:BSM_ND_PULL=0" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" "unenv:BSM_ND_PULL" \
  "env:BSM_ND_STAMPS=1" "py:scripts/solve_c5.py --orders nd --reps 1 --no-cpu-baseline"
