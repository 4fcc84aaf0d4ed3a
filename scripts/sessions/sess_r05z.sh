# round 5, session z: C1 SpMV kernel choice for tiny row counts (wave-per-64-rows against thread-per-row)
bash scripts/gpu_session.sh r05z \
  "py:scripts/perf/c1_call_probe.py" \
  "env:BSM_SPMV_VARIANT=6" \
  "py:scripts/perf/c1_call_probe.py" \
  "profpy:c1v6:scripts/perf/c1_call_probe.py 50" \
  "unenv:BSM_SPMV_VARIANT" \
  "profpy:c1v0:scripts/perf/c1_call_probe.py 50"
