# round 5, session b: RP = 4 after the fix (A/B build), the default factor after the fix,
# the half-width 16-B kernels (tests, bench, PMC against the default)
P="SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,TCC_HIT_sum,TCC_MISS_sum"
bash scripts/gpu_session.sh r05b \
  "env:BSM_LIB_PATH=basic_sparse_matrix_amd/lib/libbsm_hip_rp4.so" "env:BSM_CHOL_RPW=4" \
  "tests:tests/test_gpu_solver.py::test_poisson_500_chol4_equals_chol3_f64" \
  "py:scripts/chol_rp4_debug.py --g 500 --rpw 4 --reps 1" \
  "unenv:BSM_LIB_PATH" "unenv:BSM_CHOL_RPW" \
  "tests:tests/test_gpu_solver.py" \
  "py:scripts/chol_stress.py --g 500 --reps 3 --variants 5" \
  "tests:tests/test_gpu_tiled.py" \
  "env:BSM_TILED_HALF=3" "py:bench.py --config c4 --no-cpu-baseline --no-e2e --steps 10" \
  "unenv:BSM_TILED_HALF" "pmc:c4:$P" \
  "env:BSM_TILED_HALF=2" "pmc:c4:$P:--chunks 1" \
  "env:BSM_TILED_HALF=3" "pmc:c4:$P:--chunks 1 " \
  "unenv:BSM_TILED_HALF" "tests:tests/test_gpu_distributed.py"
