# round 6, session ae: the progressive hand-off of Linv's row blocks in
# nd_factor (BSM_ND_PROG); nd tests, C5 nd prog / none / prog, stamps
bash scripts/gpu_session.sh r06ae "tests:tests/test_gpu_solver_nd.py" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "env:BSM_ND_PROG=0" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" "unenv:BSM_ND_PROG" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
