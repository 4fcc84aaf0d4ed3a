# round 6, session p: the host analysis alone on the box's CPUs, with the
# bisection's per-depth trace (BSM_ND_TRACE=2), three runs
bash scripts/perf/build_nd_order_time.sh && \
bash scripts/gpu_session.sh r06p "env:BSM_ND_TRACE=2" "cmd:scripts/perf/bin/nd_order_time 1000 192 16" \
  "cmd:scripts/perf/bin/nd_order_time 1000 192 16" "cmd:scripts/perf/bin/nd_order_time 1000 192 16"
