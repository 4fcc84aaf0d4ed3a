# round 5, session ag: nd solves by tiles on the levels with fewer fronts than CUs (forward by tile rows,
# backward by pivot tiles), one workgroup per front below that
bash scripts/gpu_session.sh r05ag \
  "tests:tests/test_gpu_solver_nd.py" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "env:BSM_ND_FWD_TILES=0" \
  "env:BSM_ND_BWD_TILES=0" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "unenv:BSM_ND_FWD_TILES" \
  "unenv:BSM_ND_BWD_TILES" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
