"""Debug driver for the blocked solve (BSM_BLK_DEBUG=1: watchdogs around each kernel)."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
if "--debug" in sys.argv:
    os.environ["BSM_BLK_DEBUG"] = "1"
import numpy as np  # noqa: E402

from basic_sparse_matrix_amd import Csr, Dense, solve  # noqa: E402
from oracle import pyoracle as orc  # noqa: E402

for g, dt in ((2, np.float32), (5, np.float32), (20, np.float32), (20, np.float64)):
    n = g * g
    rp, ci, v = orc.poisson2d(g)
    v = v.astype(dt)
    A = Csr.from_csr_arrays((n, n), rp, ci, v)
    b = orc.gen_x_cols(1004, n, 1, dtype=dt)
    ex = orc.solve(n, rp, ci, v, b, band=True)[0]
    x = solve(A, Dense.from_columns(b), order="blocked").get_col(0)
    print(g, np.linalg.norm(x - ex) / np.linalg.norm(ex), flush=True)
