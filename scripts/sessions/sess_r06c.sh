# round 6, session c: the nd tests (cache across handles, concurrent
# handles, whole-front tasks off by default), the C5 record of all three
# orders with the CPU baseline (nd scored on its own model; cold, by-value
# and warm figures), its nd kernel stats, and the default bench line
bash scripts/gpu_session.sh r06c "tests:tests/test_gpu_solver_nd.py" smoke \
  "py:scripts/solve_c5.py --orders nd,blocked,reference --reps 3" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline" \
  "py:bench.py"
