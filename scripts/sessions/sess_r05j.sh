# round 5, session j: nd leaf size (parts left unsplit) at C5
bash scripts/gpu_session.sh r05j \
  "env:BSM_ND_LEAF=64" "py:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline" \
  "env:BSM_ND_LEAF=128" "py:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline" \
  "env:BSM_ND_LEAF=512" "py:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline" \
  "env:BSM_ND_LEAF=1024" "py:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
