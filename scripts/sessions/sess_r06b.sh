# round 6, session b: (1) the nd tests with the cache's hash fix and the
# fronts zeroed beside the analysis; (2) the nd factor's whole-front tasks:
# BSM_ND_FRONT_NT = 0 (every front by tiles, round 5) / 3 / 4 (default) / 5,
# and leaf 256 at the default; (3) C4 at N = 1 with the step split into two
# rounds whose RCCL all-gathers (world 1, BSM_MULTI_SOLO_RCCL=1) run on the
# communication stream beside the next round's SpMM, against one round and
# against two rounds without the collective, one box
bash scripts/gpu_session.sh r06b "tests:tests/test_gpu_solver_nd.py" \
  "env:BSM_ND_FRONT_NT=0" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "env:BSM_ND_FRONT_NT=3" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "env:BSM_ND_FRONT_NT=5" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "unenv:BSM_ND_FRONT_NT" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "env:BSM_ND_LEAF=256" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" "unenv:BSM_ND_LEAF" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline" \
  "py:bench.py --config c4 --no-cpu-baseline" \
  "env:BSM_MULTI_SOLO_RCCL=1" "py:bench.py --config c4 --chunks 2 --no-cpu-baseline" "unenv:BSM_MULTI_SOLO_RCCL" \
  "py:bench.py --config c4 --chunks 2 --no-cpu-baseline"
