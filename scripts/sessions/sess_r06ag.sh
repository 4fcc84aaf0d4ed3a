# round 6, session ag: the nd tests with the one-vs-several right-hand sides
# case
bash scripts/gpu_session.sh r06ag "tests:tests/test_gpu_solver_nd.py"
