# round 6, session ac: final check of HEAD's library (plan-build drain guard,
# 2^31 entry guard): the whole GPU suite, smoke, the default bench, the C5 nd
# line
bash scripts/gpu_session.sh r06ac tests smoke "py:bench.py" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline"
