"""The C1 public call (1,024 x 1,024 CSR at 1 % density, f64, one RHS column:
BASELINE configs[0], the reference's own CPU-runnable case) split into its
parts: Csr.mul_dense of the Python mirror (host Dense in, host Csr out), the
C-ABI's bsm_csr_mul_dense alone, and bsm_csr_download alone. Median of 300."""
import argparse
import ctypes
import json
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402

from basic_sparse_matrix_amd import Csr, Dense, _lib  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("calls", type=int, nargs="?", default=300)
N = ap.parse_args().calls

rng = np.random.default_rng(1000)
n = 1024
mask = rng.random((n, n)) < 0.01
rows, cols = np.nonzero(mask)
rp = np.concatenate([[0], np.cumsum(np.bincount(rows, minlength=n))]).astype(np.uint64)
a = Csr.from_csr_arrays((n, n), rp, cols.astype(np.uint64), rng.uniform(0.5, 1.5, rows.size))
xcols = [rng.uniform(-1, 1, n)]
xd = Dense.from_columns(xcols)
for _ in range(20):
    a.mul_dense(xd)
out = {"nnz": int(rows.size)}
ts = []
for _ in range(N):
    t0 = time.perf_counter()
    a.mul_dense(xd)
    ts.append(time.perf_counter() - t0)
out["public_call_ms"] = round(1e3 * float(np.median(ts)), 4)

lib = _lib.load()
h_a = a._device().handle
ptrs = (ctypes.c_void_p * 1)(xcols[0].ctypes.data)
t_mul, t_dl = [], []
onnz = ctypes.c_uint64()
for _ in range(N):
    h = ctypes.c_void_p()
    t0 = time.perf_counter()
    assert lib.bsm_csr_mul_dense(h_a, 1, n, ptrs, ctypes.byref(h)) == 0
    t1 = time.perf_counter()
    lib.bsm_csr_shape(h, None, None, ctypes.byref(onnz), None)
    orp = np.empty(n + 1, np.uint64)
    oci = np.empty(onnz.value, np.uint64)
    ov = np.empty(onnz.value, np.float64)
    t2 = time.perf_counter()
    assert lib.bsm_csr_download(h, orp.ctypes.data_as(ctypes.c_void_p), oci.ctypes.data_as(ctypes.c_void_p),
                                ov.ctypes.data_as(ctypes.c_void_p)) == 0
    t3 = time.perf_counter()
    lib.bsm_csr_free(h)
    t_mul.append(t1 - t0)
    t_dl.append(t3 - t2)
out["bsm_csr_mul_dense_ms"] = round(1e3 * float(np.median(t_mul)), 4)
out["bsm_csr_download_ms"] = round(1e3 * float(np.median(t_dl)), 4)
out["out_nnz"] = int(onnz.value)
print(json.dumps(out), flush=True)
