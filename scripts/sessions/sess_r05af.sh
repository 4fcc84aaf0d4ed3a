# round 5, session af: nd forward solve by tile rows (one wave per node, tile row, column; flags per pivot tile)
bash scripts/gpu_session.sh r05af \
  "tests:tests/test_gpu_solver_nd.py" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "env:BSM_ND_FWD_TILES=0" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "unenv:BSM_ND_FWD_TILES" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
