#!/usr/bin/env python3
"""C5: 2D 5-point Poisson (g x g grid, natural ordering), solve(A, b) on the
GPU through the reference API (lib.rs:11-24). Prints wall time and accuracy;
run under `rocprofv3 --kernel-trace --stats` for the per-kernel breakdown
(band_chol / band_forward / band_backward)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from basic_sparse_matrix_amd import Csr, Dense, solve  # noqa: E402
from oracle import pyoracle as orc  # noqa: E402  (input generation + check only)

ap = argparse.ArgumentParser()
ap.add_argument("--g", type=int, default=1000)
ap.add_argument("--dtype", default="f64")
ap.add_argument("--reps", type=int, default=1)
ap.add_argument("--order", default="reference", choices=["reference", "blocked"])
args = ap.parse_args()
dt = np.float64 if args.dtype == "f64" else np.float32
g = args.g
n = g * g
rp, ci, v = orc.poisson2d(g)
x_true = orc.gen_x_cols(1002, n, 1)[0]
rows = np.repeat(np.arange(n), np.diff(rp.astype(np.int64)))
b = np.zeros(n)
np.add.at(b, rows, v * x_true[ci.astype(np.int64)])
A = Csr.from_csr_arrays((n, n), rp, ci, v.astype(dt))
B = Dense.from_columns([b.astype(dt)])
for r in range(args.reps):
    t0 = time.perf_counter()
    x = solve(A, B, order=args.order).get_col(0)
    t = time.perf_counter() - t0
    rel = np.linalg.norm(x.astype(np.float64) - x_true) / np.linalg.norm(x_true)
    print(f"C5 g={g} N={n} {args.dtype} order={args.order}: solve wall {t:.3f} s (incl. H2D/D2H), rel err vs x_true {rel:.3e}", flush=True)
