# round 6, session v: the forward solve folded into the factor's diagonal
# tiles (one right-hand side, BSM_ND_FOLD); nd tests, C5 nd fold / no fold
# / fold, kernel stats
bash scripts/gpu_session.sh r06v "tests:tests/test_gpu_solver_nd.py" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "env:BSM_ND_FOLD=0" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" "unenv:BSM_ND_FOLD" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
