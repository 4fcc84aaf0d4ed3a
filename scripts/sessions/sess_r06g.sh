# round 6, session g: the children's update blocks pulled into the parent's
# nd_factor tiles (no nd_extend2 launches); nd tests (same bits against
# BSM_ND_PULL=0), the C5 nd line pull / push / pull, the kernel stats and
# the per-level stamps of the pull
bash scripts/gpu_session.sh r06g "tests:tests/test_gpu_solver_nd.py" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "env:BSM_ND_PULL=0" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" "unenv:BSM_ND_PULL" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline" \
  "env:BSM_ND_STAMPS=1" "py:scripts/solve_c5.py --orders nd --reps 2 --no-cpu-baseline"
