# round 6, session z: the whole GPU suite, smoke and the default bench at
# HEAD (pull with descriptors, A's entries pulled, forward folded); the C5
# record of all three orders with the CPU baseline; the nd kernel stats
bash scripts/gpu_session.sh r06z tests smoke "py:bench.py" \
  "py:scripts/solve_c5.py --orders nd,blocked,reference --reps 3" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
