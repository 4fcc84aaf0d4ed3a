# round 5, session d: BSM_C5_SPLITSTAGE measured once (C5 factor, 500^2 bits); L2 hit rate of the C4 kernel
# against the rows each XCD holds (BSM_TILED_RW sweep)
P="SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,TCC_HIT_sum,TCC_MISS_sum"
bash scripts/gpu_session.sh r05d \
  "env:BSM_LIB_PATH=basic_sparse_matrix_amd/lib/libbsm_hip_split.so" \
  "py:scripts/chol_stress.py --g 500 --reps 3" \
  "py:scripts/solve_c5.py --orders reference --reps 1 --no-cpu-baseline" \
  "unenv:BSM_LIB_PATH" \
  "py:scripts/solve_c5.py --orders reference --reps 1 --no-cpu-baseline" \
  "env:BSM_TILED_RW=100" "pmc:c4:$P:--chunks 1" \
  "env:BSM_TILED_RW=60" "pmc:c4:$P:--chunks 1 " \
  "env:BSM_TILED_RW=30" "pmc:c4:$P:--chunks 1  "
