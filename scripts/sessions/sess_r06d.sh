# round 6, session d: (1) nd_factor's per-level cycle stamps (BSM_ND_STAMPS=1,
# the diagnostic instantiation) and the host analysis's phases inside the
# solve (BSM_ND_TRACE=1) at C5; (2) C4's kernel stats under rocprofv3 and its
# PMC traffic passes (FETCH_SIZE, WRITE_SIZE, and FETCH_SIZE with every gather
# on X row 0 for the stream's calibration), for this round's profiles
bash scripts/gpu_session.sh r06d \
  "env:BSM_ND_STAMPS=1" "env:BSM_ND_TRACE=1" "py:scripts/solve_c5.py --orders nd --reps 2 --no-cpu-baseline" \
  "unenv:BSM_ND_STAMPS" "unenv:BSM_ND_TRACE" \
  "prof:c4" \
  "pmc:c4:FETCH_SIZE" "pmc:c4:WRITE_SIZE" \
  "env:BSM_TILED_PROBE_MASK=0" "pmc:c4:FETCH_SIZE:--chunks 1" "unenv:BSM_TILED_PROBE_MASK"
