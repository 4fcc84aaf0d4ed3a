# round 6, session j: the pull's phases under BSM_ND_STAMPS (diagnostic)
bash scripts/gpu_session.sh r06j "env:BSM_ND_STAMPS=1" "py:scripts/solve_c5.py --orders nd --reps 1 --no-cpu-baseline"
