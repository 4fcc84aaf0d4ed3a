# round 5, session v: HEAD validation -- the whole GPU suite, smoke, C5 (all three orders, with the
# CPU baseline), rocprofv3 kernel stats of the nd solve, the default bench line
bash scripts/gpu_session.sh r05v "tests" "smoke" \
  "py:scripts/solve_c5.py --orders nd,blocked,reference --reps 2" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline" \
  "py:bench.py"
