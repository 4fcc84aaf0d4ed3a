# round 6, session u: the nd tests with the poisoned fronts on irregular
# trees (random graph, disconnected blocks, 3-D mesh; leaves 4 / 16 / 64)
bash scripts/gpu_session.sh r06u "tests:tests/test_gpu_solver_nd.py"
