# round 5, session ae: C4 bench A/B on one box -- HEAD's library against b55c510's (the round's earlier HEAD
# validation, 180.3 ms): is the 204 ms of session ad the box or the code?
bash scripts/gpu_session.sh r05ae \
  "py:bench.py --no-cpu-baseline --no-e2e" \
  "env:BSM_LIB_PATH=basic_sparse_matrix_amd/lib/ab/libbsm_hip_b55c510.so" \
  "py:bench.py --no-cpu-baseline --no-e2e" \
  "unenv:BSM_LIB_PATH" \
  "py:bench.py --no-cpu-baseline --no-e2e"
