# round 5, session ac: nd extend-add of both children in one launch per level
bash scripts/gpu_session.sh r05ac \
  "tests:tests/test_gpu_solver_nd.py" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "env:BSM_ND_EXT_MERGE=0" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "unenv:BSM_ND_EXT_MERGE" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
