#!/usr/bin/env python3
"""A/B timing of the SpMM column-panel schedule at several panel widths in
ONE process, interleaved rounds; every width is checked bit-identical to the
one-pass kernel. C4 shape by default (10M x 10M, 1000 nnz/row, k = 32)."""
import argparse
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from basic_sparse_matrix_amd import _lib  # noqa: E402
from basic_sparse_matrix_amd.device import DeviceCsrBlock, gen_dense  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--rows", type=int, default=10_000_000)
ap.add_argument("--cols", type=int, default=10_000_000)
ap.add_argument("--nnz-row", type=int, default=1000)
ap.add_argument("--widths", default="0,2000000,1000000,500000")
ap.add_argument("--rounds", type=int, default=3)
args = ap.parse_args()
k = 32
blk = DeviceCsrBlock.generate(1000, 0, args.rows, args.cols, _lib.ROWLEN_CONST, args.nnz_row, args.nnz_row)
x = gen_dense(1001, 0, args.cols, k)
widths = [int(w) for w in args.widths.split(",")]
plans, ys, times = {}, {}, {}
for w in widths:
    t0 = time.perf_counter()
    got = blk.plan(k, w)
    torch.cuda.synchronize()
    print(f"width {w}: plan {got} in {(time.perf_counter() - t0) * 1e3:.1f} ms", flush=True)
    plans[w] = (blk.panel_cols, blk.seg)
    ys[w] = torch.empty((args.rows, k), dtype=torch.float64, device="cuda")
    times[w] = []
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for r in range(args.rounds + 1):
    for w in widths:
        blk.panel_cols, blk.seg = plans[w]
        e0.record()
        blk.spmm(x, ys[w])
        e1.record()
        torch.cuda.synchronize()
        if r > 0:
            times[w].append(e0.elapsed_time(e1))
ref = ys[widths[0]]
b_alg = 8 * (args.rows + 1) + 12 * blk.nnz + 8 * args.cols * k + 8 * args.rows * k
for w in widths:
    same = bool(torch.equal(ys[w].view(torch.int64), ref.view(torch.int64)))
    t = np.array(times[w])
    print(f"width {w}: median {np.median(t):.3f} ms min {t.min():.3f} ms  B_alg {b_alg / np.median(t) / 1e6:.1f} GB/s"
          f"  gather {blk.nnz * k * 8 / np.median(t) / 1e6:.1f} GB/s  bit-identical-to-{widths[0]}: {same}", flush=True)
