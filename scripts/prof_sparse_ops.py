#!/usr/bin/env python3
"""Profile helper: the reference benches' add_sparse / mul_sparse shapes
(1000 x 1000 u32, e random inserts per operand), a few calls each."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from basic_sparse_matrix_amd.device import csr_from_device_inserts, gen_insert_stream  # noqa: E402

e = int(sys.argv[1]) if len(sys.argv) > 1 else 900_000
op = sys.argv[2] if len(sys.argv) > 2 else "add"
a = csr_from_device_inserts((1000, 1000), *gen_insert_stream(1000, e, 1000, 1000, 255, np.uint32))
b = csr_from_device_inserts((1000, 1000), *gen_insert_stream(1001, e, 1000, 1000, 255, np.uint32))
for _ in range(5):
    t0 = time.perf_counter()
    c = a.add_sparse(b) if op == "add" else a.mul_sparse(b)
    print(f"{op} e={e}: {1e3 * (time.perf_counter() - t0):.2f} ms, out nnz {c.get_nnz()}", flush=True)
