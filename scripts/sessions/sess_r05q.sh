# round 5, session q: nd factor at two workgroups per CU again, unrolled solves
bash scripts/gpu_session.sh r05q \
  "tests:tests/test_gpu_solver_nd.py" \
  "env:BSM_ND_TRACE=1" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
