# round 5, session e: the whole GPU suite after the solver-kernel retirement; C5 both orders at HEAD
bash scripts/gpu_session.sh r05e \
  "tests" \
  "smoke" \
  "c5"
