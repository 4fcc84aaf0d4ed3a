# round 5, session c: half-width 16-B kernels with X split into two half tables
P="SQ_WAVE_CYCLES,SQ_BUSY_CYCLES,SQ_WAIT_ANY,SQ_WAIT_INST_ANY,SQ_ACTIVE_INST_ANY,SQ_WAIT_INST_LDS,SQ_LDS_BANK_CONFLICT,SQ_LDS_IDX_ACTIVE,TCC_HIT_sum,TCC_MISS_sum"
B="--config c4 --no-cpu-baseline --no-e2e --steps 10"
bash scripts/gpu_session.sh r05c \
  "tests:tests/test_gpu_tiled.py" \
  "env:BSM_TILED_HALF=3" "py:bench.py $B" \
  "env:BSM_TILED_PSHIFT=13" "py:bench.py $B" "unenv:BSM_TILED_PSHIFT" \
  "pmc:c4:$P" \
  "env:BSM_TILED_HALF=2" "py:bench.py $B" \
  "unenv:BSM_TILED_HALF" "py:bench.py $B"
