# round 6, session w: the folded forward solve, measured again with
# scripts/solve_c5.py reporting it as folded (no forward fraction of its
# own): C5 nd fold / no fold / fold, kernel stats, the C5 record of the nd
# order with the CPU baseline
bash scripts/gpu_session.sh r06w \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "env:BSM_ND_FOLD=0" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" "unenv:BSM_ND_FOLD" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
