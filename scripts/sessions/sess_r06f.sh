# round 6, session f: the lagged order of the tiles below a diagonal
# (BSM_ND_LAG, nd_layout) and the levels' lists built on threads; nd tests,
# then the C5 nd line at lags 0 (round-5 order), 128, 512 (default) and 1024
bash scripts/gpu_session.sh r06f "tests:tests/test_gpu_solver_nd.py" \
  "env:BSM_ND_LAG=0" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "env:BSM_ND_LAG=128" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "env:BSM_ND_LAG=1024" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "unenv:BSM_ND_LAG" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "env:BSM_ND_STAMPS=1" "py:scripts/solve_c5.py --orders nd --reps 2 --no-cpu-baseline"
