# round 5, session i: nd solve with the band-window root cut and pinned staging: tests, C5 cold/warm,
# rocprofv3 kernel stats of the nd C5 solve
bash scripts/gpu_session.sh r05i \
  "tests:tests/test_gpu_solver_nd.py" \
  "env:BSM_ND_TRACE=1" \
  "py:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 2 --no-cpu-baseline"
