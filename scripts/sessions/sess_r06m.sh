# round 6, session m: the cold path with and without the fronts' zeroing on
# the helper stream (BSM_ND_PREZERO), now that the layout is ~6 ms
bash scripts/gpu_session.sh r06m \
  "env:BSM_ND_TRACE=1" "py:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline" \
  "env:BSM_ND_PREZERO=0" "py:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline" "unenv:BSM_ND_PREZERO" \
  "py:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline" \
  "env:BSM_ND_PREZERO=0" "py:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
