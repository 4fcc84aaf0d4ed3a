# round 6, session a: the nd plan cache across handles (pattern key on the
# device), nd_forward_tiles restructured, the analysis on per-part graphs;
# the whole GPU suite, smoke, the C5 nd record with its own model and its
# rocprofv3 kernel stats, the host analysis A/B against round 5, and the
# ss_add phase times (BSM_SS_DEBUG=3)
bash scripts/gpu_session.sh r06a tests smoke \
  "py:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline" \
  "cmd:bash scripts/perf/nd_analysis_ab.sh" \
  "env:BSM_SS_DEBUG=3" "py:bench.py --ref-benches ss_add"
