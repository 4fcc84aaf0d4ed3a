# round 5, session x: the C1 public call split, and its kernels / HIP calls; the chol5 delay knob's effect
bash scripts/gpu_session.sh r05x \
  "py:scripts/perf/c1_call_probe.py" \
  "py:scripts/perf/chol5_delay_probe.py 100" \
  "cmd:rocprofv3 --kernel-trace --hip-runtime-trace --stats -d gpurun_out/c1_trace_r05x -o run --output-format csv -- python scripts/perf/c1_call_probe.py 50"
