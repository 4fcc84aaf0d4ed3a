# round 6, session ab: the leaf size at C5 on the current pipeline
# (BSM_ND_LEAF 96 / 128 / 160 / 192 (default) / 256)
bash scripts/gpu_session.sh r06ab \
  "env:BSM_ND_LEAF=96" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "env:BSM_ND_LEAF=128" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "env:BSM_ND_LEAF=160" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "unenv:BSM_ND_LEAF" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "env:BSM_ND_LEAF=256" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline"
