# round 6, session i: the pull with both children's descriptors and bounds
# loaded up front; nd tests, C5 nd (pull, push), stamps
bash scripts/gpu_session.sh r06i "tests:tests/test_gpu_solver_nd.py" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "env:BSM_ND_PULL=0" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" "unenv:BSM_ND_PULL" \
  "env:BSM_ND_STAMPS=1" "py:scripts/solve_c5.py --orders nd --reps 1 --no-cpu-baseline"
