# round 5, session ak: nd solve kernels with nd_factor's ticket pattern: the combination probe, then the nd tests
bash scripts/gpu_session.sh r05ak \
  "py:scripts/perf/nd_tiles_probe.py --limit 40" \
  "tests:tests/test_gpu_solver_nd.py"
