"""Wall time of cholesky_decomp (band_chol5) at several BSM_CHOL5_DELAY
values: shows that the stress knob the completion tests use really slows the
late side (tests/test_gpu_solver.py::test_chol5_completion_with_late_waves_vs_oracle)."""
import argparse
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from basic_sparse_matrix_amd import Csr  # noqa: E402


def poisson2d(g):
    n = g * g
    rows, cols, vals = [], [], []
    for i in range(n):
        r, c = divmod(i, g)
        for j, v in ((i - g, -1.0), (i - 1, -1.0), (i, 4.0), (i + 1, -1.0), (i + g, -1.0)):
            if 0 <= j < n and (j == i or abs(j - i) == g or (j // g == r)):
                rows.append(i); cols.append(j); vals.append(v)
    rp = np.zeros(n + 1, np.uint64)
    np.add.at(rp, np.array(rows) + 1, 1)
    return n, np.cumsum(rp).astype(np.uint64), np.array(cols, np.uint64), np.array(vals)


ap = argparse.ArgumentParser()
ap.add_argument("g", type=int, nargs="?", default=100)
g = ap.parse_args().g
n, rp, ci, v = poisson2d(g)
A = Csr.from_csr_arrays((n, n), rp, ci, v)
A.cholesky_decomp()  # warm
out = {"g": g, "row_blocks": (n + 15) // 16}
for d in (0, 8, -8, 32):
    os.environ["BSM_CHOL5_DELAY"] = str(d)
    t = time.perf_counter()
    A.cholesky_decomp()
    out[f"ms_delay_{d}"] = round((time.perf_counter() - t) * 1e3, 2)
os.environ.pop("BSM_CHOL5_DELAY")
print(json.dumps(out))
