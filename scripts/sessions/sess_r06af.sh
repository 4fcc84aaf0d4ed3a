# round 6, session af: the library rebuilt from HEAD after the dropped A/B:
# the whole GPU suite, smoke, the C5 nd line
bash scripts/gpu_session.sh r06af tests smoke "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline"
