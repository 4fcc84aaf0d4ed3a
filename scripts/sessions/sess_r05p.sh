# round 5, session p: nd plan A/B: corner BFS roots after the band cut (default) vs the far-vertex search
bash scripts/gpu_session.sh r05p \
  "env:BSM_ND_TRACE=1" \
  "profpy:c5nd_hint:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline" \
  "env:BSM_ND_BANDHINT=0" \
  "profpy:c5nd_search:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
