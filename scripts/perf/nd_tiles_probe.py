"""Which nd solve kernel combination finishes on small systems: each run in
its own process under a time limit (a stuck hand-off ends as a timeout error
or the limit, not as a hung session)."""
import argparse
import os
import subprocess
import sys

ap = argparse.ArgumentParser()
ap.add_argument("--limit", type=int, default=40)
args = ap.parse_args()
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
CODE = r'''
import sys, time
sys.path.insert(0, %r)
import numpy as np
from basic_sparse_matrix_amd import Csr, Dense, solve
a = Csr.from_data([[4.0, 1.0, 0.0, 0.0], [1.0, 4.0, 1.0, 0.0], [0.0, 1.0, 4.0, 1.0], [0.0, 0.0, 1.0, 4.0]], dtype=np.float64)
t = time.time()
x = solve(a, Dense.from_columns([np.array([1.0, 2.0, 3.0, 4.0])]), order="nd").get_col(0)
print("4x4", np.asarray(x).tolist(), round(time.time() - t, 3), flush=True)
g = 30
n = g * g
idx = np.arange(n).reshape(g, g)
rows, cols, vals = [idx.ravel()], [idx.ravel()], [np.full(n, 4.5)]
for ax in range(2):
    p = np.take(idx, range(g - 1), axis=ax).ravel(); q = np.take(idx, range(1, g), axis=ax).ravel()
    rows += [p, q]; cols += [q, p]; vals += [np.full(p.size, -1.0)] * 2
r, c, v = np.concatenate(rows), np.concatenate(cols), np.concatenate(vals)
o = np.lexsort((c, r)); r, c, v = r[o], c[o], v[o]
rp = np.concatenate([[0], np.cumsum(np.bincount(r, minlength=n))]).astype(np.uint64)
A = Csr.from_csr_arrays((n, n), rp, c.astype(np.uint64), v)
b = np.linspace(-1, 1, n)
t = time.time()
x = np.asarray(solve(A, Dense.from_columns([b]), order="nd").get_col(0))
res = np.zeros(n); np.add.at(res, r, v * x[c]); print("g30 residual", float(np.linalg.norm(res - b)), round(time.time() - t, 3), flush=True)
''' % ROOT
for fwd, bwd in (("0", "0"), ("1", "0"), ("0", "1"), ("1", "1")):
    env = dict(os.environ, BSM_ND_FWD_TILES=fwd, BSM_ND_BWD_TILES=bwd)
    try:
        p = subprocess.run([sys.executable, "-c", CODE], env=env, capture_output=True, text=True, timeout=args.limit)
        out = (p.stdout + p.stderr[-400:]).strip().replace("\n", " | ")
        print(f"fwd_tiles={fwd} bwd_tiles={bwd}: rc={p.returncode} {out}", flush=True)
    except subprocess.TimeoutExpired:
        print(f"fwd_tiles={fwd} bwd_tiles={bwd}: TIMEOUT after {args.limit} s", flush=True)
        break
