# round 6, session a: the nd plan cache across handles (pattern key on the
# device), nd_forward_tiles restructured, the honest nd model in solve_c5.py
bash scripts/gpu_session.sh r06a "tests:tests/test_gpu_solver_nd.py" \
  "py:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
