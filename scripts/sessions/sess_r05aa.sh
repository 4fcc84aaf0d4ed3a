# round 5, session aa: spmv_thread for few short rows + small-result host copy: SpMM / build / config tests, C1 probe and bench
bash scripts/gpu_session.sh r05aa \
  "tests:tests/test_gpu_spmm.py tests/test_gpu_build.py tests/test_gpu_configs.py tests/test_gpu_sparse_ops.py" \
  "py:scripts/perf/c1_call_probe.py" \
  "bench:c1" \
  "profpy:c1:scripts/perf/c1_call_probe.py 50"
