# round 5, session al: C5 nd with the solves by tiles on the small levels (hybrid), against both off
bash scripts/gpu_session.sh r05al \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "env:BSM_ND_FWD_TILES=0" \
  "env:BSM_ND_BWD_TILES=0" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "unenv:BSM_ND_FWD_TILES" \
  "unenv:BSM_ND_BWD_TILES" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
