#!/usr/bin/env python3
"""A/B timing of SpMM kernel variants (BSM_SPMM_VARIANT) in ONE process,
interleaved rounds (cdna_hip_programming.md §5.4 rule 24). C4 shape by
default (10M x 10M, 1000 nnz/row, k = 32, f64); --rows scales it down."""
import argparse
import os
import sys

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
ap.add_argument("--k", type=int, default=32)
ap.add_argument("--variants", default="1,2,3,4")
ap.add_argument("--rounds", type=int, default=3)
ap.add_argument("--env", default="BSM_SPMM_VARIANT", help="environment variable the variants set")
args = ap.parse_args()

blk = DeviceCsrBlock.generate(1000, 0, args.rows, args.cols, _lib.ROWLEN_CONST, args.nnz_row, args.nnz_row)
x = gen_dense(1001, 0, args.cols, args.k)
ys = {}
times = {}
variants = [int(v) for v in args.variants.split(",")]
for v in variants:
    ys[v] = torch.empty((args.rows, args.k), dtype=torch.float64, device="cuda")
    times[v] = []
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for r in range(args.rounds + 1):
    for v in variants:
        os.environ[args.env] = str(v)
        e0.record()
        blk.spmm(x, ys[v])
        e1.record()
        torch.cuda.synchronize()
        if r > 0:
            times[v].append(e0.elapsed_time(e1))
ref = ys[variants[0]]
nnz = blk.nnz
b_alg = 8 * (args.rows + 1) + 12 * nnz + 8 * args.cols * args.k + 8 * args.rows * args.k
for v in variants:
    same = bool(torch.equal(ys[v].view(torch.int64), ref.view(torch.int64)))
    t = np.array(times[v])
    print(f"variant {v}: median {np.median(t):.3f} ms min {t.min():.3f} ms  B_alg {b_alg / np.median(t) / 1e6:.1f} GB/s"
          f"  gather {nnz * args.k * 8 / np.median(t) / 1e6:.1f} GB/s  bit-identical-to-{variants[0]}: {same}",
          flush=True)
