# round 5, session h: host analysis of solve(order="nd") on the GPU box's cores (thread counts,
# parallel BFS on/off, start-vertex hints), then C5 with the plan cached on the handle
T=scripts/perf/bin/nd_order_time
bash scripts/gpu_session.sh r05h \
  "cmd:$T 1000 256 1" "cmd:$T 1000 256 16" \
  "env:BSM_ND_PBFS=4" "cmd:$T 1000 256 16" \
  "env:BSM_ND_PBFS=8" "cmd:$T 1000 256 16" \
  "env:BSM_ND_PBFS=16" "cmd:$T 1000 256 16" \
  "unenv:BSM_ND_PBFS" \
  "env:BSM_ND_HINT=0" "cmd:$T 1000 256 16" "env:BSM_ND_HINT=2" "cmd:$T 1000 256 16" "unenv:BSM_ND_HINT" \
  "tests:tests/test_gpu_solver_nd.py" \
  "py:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
