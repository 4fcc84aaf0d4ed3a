#!/usr/bin/env python3
"""Profile helper: per-call API overhead of Csr.mul_dense on the reference
bench's sd_mul shape (1000 x 1000 u32, 900k inserts, k = 10)."""
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402,F401

from basic_sparse_matrix_amd import Dense  # noqa: E402
from basic_sparse_matrix_amd.device import csr_from_device_inserts, gen_insert_stream  # noqa: E402

a = csr_from_device_inserts((1000, 1000), *gen_insert_stream(1000, 900_000, 1000, 1000, 255, np.uint32))
rng = np.random.default_rng(1)
x = Dense.from_columns([rng.integers(0, 255, 1000).astype(np.uint32) for _ in range(10)])
for _ in range(3):
    a.mul_dense(x)
ts = []
for _ in range(50):
    t0 = time.perf_counter()
    a.mul_dense(x)
    ts.append(time.perf_counter() - t0)
print(f"mul_dense per call: median {1e3 * np.median(ts):.3f} ms", flush=True)
