# round 5, session k: add/sub wave-per-row path (tests) and the reference bench suite's ss_add
bash scripts/gpu_session.sh r05k \
  "tests:tests/test_gpu_sparse_ops.py" \
  "py:bench.py --ref-benches ss_add"
