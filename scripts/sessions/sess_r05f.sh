# round 5, session f: bench lines at HEAD (C1-C4), L2 hit rates of the C1-C3 kernels (roofline_gather's
# peak model), rocprofv3 kernel stats of C4
H="TCC_HIT_sum,TCC_MISS_sum"
bash scripts/gpu_session.sh r05f \
  "py:bench.py --config c4" \
  "py:bench.py --config c3" \
  "py:bench.py --config c2" \
  "py:bench.py --config c1" \
  "pmc:c3:$H" "pmc:c2:$H" "pmc:c1:$H" \
  "prof:c4:--steps 5" \
  "tests:tests/test_gpu_distributed.py tests/test_gpu_multi.py"
