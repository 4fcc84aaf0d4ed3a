# round 6, session l: the tiles no A entry lands in start from zero (no
# zeroing, no read; BSM_ND_ZSKIP); nd tests, C5 nd zskip / no zskip /
# zskip, the kernel stats, the cold path's phases
bash scripts/gpu_session.sh r06l "tests:tests/test_gpu_solver_nd.py" \
  "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" \
  "env:BSM_ND_ZSKIP=0" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" "unenv:BSM_ND_ZSKIP" \
  "env:BSM_ND_TRACE=1" "py:scripts/solve_c5.py --orders nd --reps 5 --no-cpu-baseline" "unenv:BSM_ND_TRACE" \
  "profpy:c5nd:scripts/solve_c5.py --orders nd --reps 3 --no-cpu-baseline"
