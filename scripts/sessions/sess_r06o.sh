# round 6, session o: the whole GPU suite, smoke and the default bench at
# HEAD (pull, zero-skip, lag); the C5 record of all three orders with the
# CPU baseline; the nd kernel stats
bash scripts/gpu_session.sh r06o tests smoke "py:bench.py" \
  "py:scripts/solve_c5.py --orders nd,blocked,reference --reps 3" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
