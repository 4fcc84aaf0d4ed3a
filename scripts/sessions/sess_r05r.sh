# round 5, session r: nd leaf size sweep with the diagonal-first tile order
bash scripts/gpu_session.sh r05r \
  "env:BSM_ND_LEAF=128" "py:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline" \
  "env:BSM_ND_LEAF=192" "py:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline" \
  "env:BSM_ND_LEAF=320" "py:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
