# round 5, session y: small mul_dense results compacted in one workgroup with a host copy (C1 public call)
bash scripts/gpu_session.sh r05y \
  "tests:tests/test_gpu_spmm.py tests/test_gpu_build.py tests/test_gpu_configs.py" \
  "py:scripts/perf/c1_call_probe.py" \
  "env:BSM_SMALL_OUT=0" \
  "py:scripts/perf/c1_call_probe.py" \
  "unenv:BSM_SMALL_OUT" \
  "bench:c1"
