"""ctypes wrapper of the CPU ORACLE (oracle/build/libbsm_oracle.so).

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg -- never by basic_sparse_matrix_amd/. The C code
restates the reference's algorithms (see bsm_oracle.h for citations).
"""

from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "build", "libbsm_oracle.so")

ORC_OK, ORC_ERR_INCORRECT_DIMENSIONS, ORC_ERR_NON_SQUARE, ORC_ERR_PANIC, ORC_ERR_ALLOC, ORC_ERR_UNSUPPORTED = range(6)

SUFFIX = {
    np.dtype(np.float64): "f64",
    np.dtype(np.float32): "f32",
    np.dtype(np.int32): "i32",
    np.dtype(np.uint32): "u32",
    np.dtype(np.int64): "i64",
    np.dtype(np.uint64): "u64",
}

ROWLEN_CONST, ROWLEN_UNIFORM, ROWLEN_BINOMIAL = 0, 1, 2
VAL_UNIFORM, VAL_SMALLINT = 0, 1


class OracleError(RuntimeError):
    def __init__(self, code):
        super().__init__(f"oracle returned {code}")
        self.code = code


_lib = None


def build() -> str:
    subprocess.run(["make", "-s", "-C", HERE], check=True)
    return LIB


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(LIB):
            build()
        _lib = ctypes.CDLL(LIB)
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data if a.size else 0)


def _u64(a):
    return np.ascontiguousarray(a, dtype=np.uint64)


def _check(rc):
    if rc != ORC_OK:
        raise OracleError(rc)


def csr_from_inserts(rows, row, col, v):
    """Csr::insert(v[i], row[i], col[i]) for every i, then finalise
    (sparse.rs:206-250) -> (row_index u64 [rows+1], col u64, v)."""
    v = np.ascontiguousarray(v)
    dt = v.dtype
    r, c = _u64(row), _u64(col)
    n = len(v)
    out_row = np.zeros(rows + 1, dtype=np.uint64)
    out_col = np.zeros(max(1, n), dtype=np.uint64)
    out_v = np.zeros(max(1, n), dtype=dt)
    nnz = ctypes.c_uint64(0)
    fn = getattr(lib(), "orc_csr_from_inserts_" + SUFFIX[dt])
    rc = fn(ctypes.c_uint64(rows), ctypes.c_uint64(n), _p(r), _p(c), _p(v), _p(out_row), _p(out_col), _p(out_v),
            ctypes.byref(nnz))
    _check(rc)
    m = nnz.value
    return out_row, out_col[:m].copy(), out_v[:m].copy()


def mul_dense(rows, cols, row_index, col_index, v, x_cols, x_rows=None):
    """Csr::mul_dense (sparse.rs:426-446). x_cols: list of k columns."""
    v = np.ascontiguousarray(v)
    dt = v.dtype
    k = len(x_cols)
    x_rows = cols if x_rows is None else x_rows
    x = np.zeros((max(k, 1), x_rows), dtype=dt)
    for j, c in enumerate(x_cols):
        x[j, :] = c
    ri, ci = _u64(row_index), _u64(col_index)
    out_row = np.zeros(rows + 1, dtype=np.uint64)
    cap = max(1, rows * k)
    out_col = np.zeros(cap, dtype=np.uint64)
    out_v = np.zeros(cap, dtype=dt)
    nnz_out = ctypes.c_uint64(0)
    fn = getattr(lib(), "orc_mul_dense_" + SUFFIX[dt])
    rc = fn(ctypes.c_uint64(rows), ctypes.c_uint64(cols), _p(ri), ctypes.c_uint64(len(ri)), _p(ci), _p(v),
            ctypes.c_uint64(len(v)), ctypes.c_uint64(k), ctypes.c_uint64(x_rows), _p(x), ctypes.c_uint64(x_rows),
            _p(out_row), _p(out_col), _p(out_v), ctypes.byref(nnz_out))
    _check(rc)
    n = nnz_out.value
    return out_row, out_col[:n].copy(), out_v[:n].copy()


def mul_vector(rows, cols, row_index, col_index, v, rhs, out_len=None):
    v = np.ascontiguousarray(v)
    dt = v.dtype
    rhs = np.ascontiguousarray(rhs, dtype=dt)
    out_len = rows if out_len is None else out_len
    out = np.zeros(out_len, dtype=dt)
    ri, ci = _u64(row_index), _u64(col_index)
    fn = getattr(lib(), "orc_mul_vector_" + SUFFIX[dt])
    rc = fn(ctypes.c_uint64(rows), ctypes.c_uint64(cols), _p(ri), ctypes.c_uint64(len(ri)), _p(ci), _p(v),
            ctypes.c_uint64(len(v)), _p(rhs), ctypes.c_uint64(len(rhs)), _p(out), ctypes.c_uint64(out_len))
    _check(rc)
    return out


def transpose(rows, cols, row_index, col_index, v):
    v = np.ascontiguousarray(v)
    dt = v.dtype
    ri, ci = _u64(row_index), _u64(col_index)
    t_row = np.zeros(cols + 1, dtype=np.uint64)
    t_col = np.zeros(max(1, len(v)), dtype=np.uint64)
    t_v = np.zeros(max(1, len(v)), dtype=dt)
    fn = getattr(lib(), "orc_transpose_" + SUFFIX[dt])
    rc = fn(ctypes.c_uint64(rows), ctypes.c_uint64(cols), _p(ri), ctypes.c_uint64(len(ri)), _p(ci), _p(v),
            ctypes.c_uint64(len(v)), _p(t_row), _p(t_col), _p(t_v))
    _check(rc)
    n = int(t_row[cols])
    return t_row, t_col[:n].copy(), t_v[:n].copy()


def cholesky(n_rows, n_cols, row_index, col_index, v, band=False):
    """cholesky_decomp (sparse.rs:682-714): literal or band restatement."""
    v = np.ascontiguousarray(v)
    dt = v.dtype
    ri, ci = _u64(row_index), _u64(col_index)
    name = ("orc_cholesky_band_" if band else "orc_cholesky_literal_") + SUFFIX[dt]
    fn = getattr(lib(), name)
    cap = ctypes.c_uint64(0)
    null = ctypes.c_void_p(0)
    rc = fn(ctypes.c_uint64(n_rows), ctypes.c_uint64(n_cols), _p(ri), _p(ci), _p(v), null, null, null,
            ctypes.byref(cap))
    if rc not in (ORC_OK, ORC_ERR_ALLOC):
        raise OracleError(rc)
    l_row = np.zeros(n_rows + 1, dtype=np.uint64)
    l_col = np.zeros(max(1, cap.value), dtype=np.uint64)
    l_v = np.zeros(max(1, cap.value), dtype=dt)
    rc = fn(ctypes.c_uint64(n_rows), ctypes.c_uint64(n_cols), _p(ri), _p(ci), _p(v), _p(l_row), _p(l_col),
            _p(l_v), ctypes.byref(cap))
    _check(rc)
    return l_row, l_col[: cap.value].copy(), l_v[: cap.value].copy()


def _trsv(name, n, row, col, v, b_cols):
    v = np.ascontiguousarray(v)
    dt = v.dtype
    k = len(b_cols)
    b = np.zeros((max(k, 1), n), dtype=dt)
    for j, c in enumerate(b_cols):
        b[j, :] = c
    x = np.zeros((max(k, 1), n), dtype=dt)
    fn = getattr(lib(), name + SUFFIX[dt])
    rc = fn(ctypes.c_uint64(n), _p(_u64(row)), _p(_u64(col)), _p(v), ctypes.c_uint64(k), _p(b),
            ctypes.c_uint64(n), _p(x), ctypes.c_uint64(n))
    _check(rc)
    return [x[j].copy() for j in range(k)]


def forward_substitution(n, l_row, l_col, l_v, b_cols):
    return _trsv("orc_forward_substitution_", n, l_row, l_col, l_v, b_cols)


def backward_substitution(n, u_row, u_col, u_v, y_cols):
    return _trsv("orc_backward_substitution_", n, u_row, u_col, u_v, y_cols)


def solve(n, row_index, col_index, v, b_cols, band=False):
    v = np.ascontiguousarray(v)
    dt = v.dtype
    k = len(b_cols)
    b = np.zeros((max(k, 1), n), dtype=dt)
    for j, c in enumerate(b_cols):
        b[j, :] = c
    x = np.zeros((max(k, 1), n), dtype=dt)
    fn = getattr(lib(), "orc_solve_" + SUFFIX[dt])
    rc = fn(ctypes.c_uint64(n), _p(_u64(row_index)), _p(_u64(col_index)), _p(v), ctypes.c_uint64(k), _p(b),
            ctypes.c_uint64(n), _p(x), ctypes.c_uint64(n), ctypes.c_int(1 if band else 0))
    _check(rc)
    return [x[j].copy() for j in range(k)]


# ------------------------------------------------------------- generators
def gen_row_ptr(seed, rows, n_cols, kind=ROWLEN_CONST, a=10, b=10):
    rp = np.zeros(rows + 1, dtype=np.uint64)
    lib().orc_gen_row_ptr(ctypes.c_uint64(seed), ctypes.c_uint64(rows), ctypes.c_uint32(n_cols), ctypes.c_int(kind),
                          ctypes.c_uint32(a), ctypes.c_uint32(b), _p(rp))
    return rp


def gen_entries(seed, row_ptr, n_cols, value_kind=VAL_UNIFORM, r0=0, r1=None):
    rows = len(row_ptr) - 1
    r1 = rows if r1 is None else r1
    nnz = int(row_ptr[rows])
    ci = np.zeros(max(1, nnz), dtype=np.uint64)
    v = np.zeros(max(1, nnz), dtype=np.float64)
    rc = lib().orc_gen_entries(ctypes.c_uint64(seed), ctypes.c_uint64(r0), ctypes.c_uint64(r1),
                               ctypes.c_uint32(n_cols), _p(_u64(row_ptr)), ctypes.c_int(value_kind), _p(ci), _p(v))
    _check(rc)
    return ci[:nnz], v[:nnz]


def gen_csr(seed, rows, n_cols, kind=ROWLEN_CONST, a=10, b=10, value_kind=VAL_UNIFORM, dtype=np.float64):
    """Synthetic CSR per bsm_synth.h -> (row_ptr u64, col u64, vals dtype)."""
    rp = gen_row_ptr(seed, rows, n_cols, kind, a, b)
    ci, v = gen_entries(seed, rp, n_cols, value_kind)
    return rp, ci, v.astype(dtype)


def gen_x_cols(seed, n_cols, k, value_kind=VAL_UNIFORM, dtype=np.float64):
    x = np.zeros((max(k, 1), n_cols), dtype=np.float64)
    lib().orc_gen_x_colmajor(ctypes.c_uint64(seed), ctypes.c_uint64(n_cols), ctypes.c_uint64(k),
                             ctypes.c_int(value_kind), _p(x))
    return [x[j].astype(dtype) for j in range(k)]


def gen_insert_stream(seed, n, rows=1000, cols=1000, vmod=255):
    """Bench-shaped insert stream (bsm_synth.h bsm_stream_draw) -> row, col, v (u64)."""
    r = np.zeros(max(1, n), dtype=np.uint64)
    c = np.zeros(max(1, n), dtype=np.uint64)
    v = np.zeros(max(1, n), dtype=np.uint64)
    lib().orc_gen_insert_stream(ctypes.c_uint64(seed), ctypes.c_uint64(n), ctypes.c_uint64(rows),
                                ctypes.c_uint64(cols), ctypes.c_uint64(vmod), _p(r), _p(c), _p(v))
    return r[:n], c[:n], v[:n]


def poisson2d(g):
    n = g * g
    nnz = lib().orc_gen_poisson2d
    nnz.restype = ctypes.c_uint64
    cap = 5 * n
    rp = np.zeros(n + 1, dtype=np.uint64)
    ci = np.zeros(cap, dtype=np.uint64)
    v = np.zeros(cap, dtype=np.float64)
    m = nnz(ctypes.c_uint64(g), _p(rp), _p(ci), _p(v))
    return rp, ci[:m].copy(), v[:m].copy()


def csr_from_coo(rows, cols, row, col, v):
    """From<COO<T>> for Csr<T> (sparse.rs:56-66) -> (row_index, col, v)."""
    v = np.ascontiguousarray(v)
    dt = v.dtype
    r, c = _u64(row), _u64(col)
    n = len(v)
    out_row = np.zeros(rows + 1, dtype=np.uint64)
    out_col = np.zeros(max(1, n), dtype=np.uint64)
    out_v = np.zeros(max(1, n), dtype=dt)
    nnz = ctypes.c_uint64(0)
    fn = getattr(lib(), "orc_csr_from_coo_" + SUFFIX[dt])
    rc = fn(ctypes.c_uint64(rows), ctypes.c_uint64(cols), ctypes.c_uint64(n), _p(r), _p(c), _p(v), _p(out_row),
            _p(out_col), _p(out_v), ctypes.byref(nnz))
    _check(rc)
    m = nnz.value
    return out_row, out_col[:m].copy(), out_v[:m].copy()


def _sparse_op(name, sub, a, b, cap):
    (ar, ac, arp, aci, av), (br, bc, brp, bci, bv) = a, b
    av = np.ascontiguousarray(av)
    dt = av.dtype
    bv = np.ascontiguousarray(bv, dtype=dt)
    rows_out = ar
    out_row = np.zeros(rows_out + 1, dtype=np.uint64)
    out_col = np.zeros(max(1, cap), dtype=np.uint64)
    out_v = np.zeros(max(1, cap), dtype=dt)
    nnz = ctypes.c_uint64(0)
    fn = getattr(lib(), name + SUFFIX[dt])
    args = [ctypes.c_uint64(ar), ctypes.c_uint64(ac), _p(_u64(arp)), _p(_u64(aci)), _p(av), ctypes.c_uint64(br),
            ctypes.c_uint64(bc), _p(_u64(brp)), _p(_u64(bci)), _p(bv), _p(out_row), _p(out_col), _p(out_v),
            ctypes.byref(nnz)]
    rc = fn(ctypes.c_int(sub), *args) if sub is not None else fn(*args)
    _check(rc)
    m = nnz.value
    return out_row, out_col[:m].copy(), out_v[:m].copy()


def add_sparse(a, b):
    """Csr::add_sparse (sparse.rs:484-540). a, b: (rows, cols, row_index, col, v)."""
    return _sparse_op("orc_addsub_sparse_", 0, a, b, len(a[4]) + len(b[4]))


def sub_sparse(a, b):
    """Csr::sub_sparse (sparse.rs:542-599)."""
    return _sparse_op("orc_addsub_sparse_", 1, a, b, len(a[4]) + len(b[4]))


def mul_sparse(a, b):
    """Csr::mul_sparse (sparse.rs:601-635): dims (a.rows, b.cols)."""
    return _sparse_op("orc_mul_sparse_", None, a, b, a[0] * b[1])
