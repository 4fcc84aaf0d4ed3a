# round 6, session h: the pull with one round trip of loads per child (rows
# per lane, columns wave-uniform); nd tests, C5 nd pull / push / pull, the
# kernel stats, the stamps
bash scripts/gpu_session.sh r06h "tests:tests/test_gpu_solver_nd.py" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "env:BSM_ND_PULL=0" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" "unenv:BSM_ND_PULL" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline" \
  "env:BSM_ND_STAMPS=1" "py:scripts/solve_c5.py --orders nd --reps 2 --no-cpu-baseline"
