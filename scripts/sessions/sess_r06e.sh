# round 6, session e: the plan's device buffer and page-locked staging
# allocated on the helper thread during the layout (cold path); nd tests and
# the C5 nd line with the analysis phases (BSM_ND_TRACE=1)
bash scripts/gpu_session.sh r06e "tests:tests/test_gpu_solver_nd.py" \
  "env:BSM_ND_TRACE=1" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline"
