# round 5, session w: band_chol5 completion under late store waves / late wave 0
bash scripts/gpu_session.sh r05w \
  "tests:tests/test_gpu_solver.py"
