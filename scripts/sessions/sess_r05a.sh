bash scripts/gpu_session.sh r05a \
  "tests:tests/test_gpu_tiled.py" \
  "env:BSM_TILED_HALF=2" "py:bench.py --config c4 --no-cpu-baseline --no-e2e --steps 10" \
  "unenv:BSM_TILED_HALF" "py:bench.py --config c4 --no-cpu-baseline --no-e2e --steps 10" \
  "env:BSM_TILED_HALF=2" "py:bench.py --config c4 --no-cpu-baseline --no-e2e --steps 10" \
  "unenv:BSM_TILED_HALF" \
  "env:BSM_LIB_PATH=basic_sparse_matrix_amd/lib/libbsm_hip_rp4old.so" "py:scripts/chol_rp4_debug.py --g 500 --rpw 4 --reps 2" \
  "env:BSM_LIB_PATH=basic_sparse_matrix_amd/lib/libbsm_hip_rp4.so" "py:scripts/chol_rp4_debug.py --g 500 --rpw 4 --reps 2" \
  "unenv:BSM_LIB_PATH" "py:scripts/chol_stress.py --g 500 --reps 3 --variants 5" \
  "env:BSM_TILED_HALF=2" "tests:tests/test_gpu_configs.py::test_c4_full_size_two_schedules_and_oracle_samples" \
  "unenv:BSM_TILED_HALF" "tests:tests/test_gpu_distributed.py"
