# round 5, session l: the whole GPU suite, smoke and the default bench line at HEAD
bash scripts/gpu_session.sh r05l "tests" "smoke" "py:bench.py"
