# round 5, session ao: smoke and the solver GPU tests at the final HEAD
bash scripts/gpu_session.sh r05ao "smoke" \
  "tests:tests/test_gpu_solver_nd.py tests/test_gpu_solver.py tests/test_gpu_solver_blocked.py"
