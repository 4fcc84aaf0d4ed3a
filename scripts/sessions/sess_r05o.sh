# round 5, session o: nd factor A/B on one box: plain staging vs pipelined loads (BSM_ND_PIPE=1)
bash scripts/gpu_session.sh r05o \
  "tests:tests/test_gpu_solver_nd.py" "env:BSM_ND_PIPE=1" "tests:tests/test_gpu_solver_nd.py" "unenv:BSM_ND_PIPE" \
  "profpy:c5nd_plain:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline" \
  "env:BSM_ND_PIPE=1" \
  "profpy:c5nd_pipe:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
