"""GPU parity of device construction from an insert sequence (Csr::insert
then finalise, src/sparse.rs:206-250) and of mul_dense on
the reference bench's input shape (benches/sparse_dense_mul.rs:8-35: u32,
random insert order, the running-max row rule piling almost every entry into
the last row), which takes the nnz-balanced integer SpMM.

Expected values come from the CPU oracle (oracle/), pinned by
tests/test_oracle_golden.py against the reference's own unit tests. The bar
is bit-exact row_ptr / col_idx / values.
"""

import numpy as np
import pytest

from basic_sparse_matrix_amd import Csr, Dense, Panic
from test_gpu_spmm import assert_csr_bits
from test_oracle_golden import from_data_inserts

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("name", ["example_mat_0", "example_mat_1", "example_mat_2", "csr_with_empty_row_top",
                                  "csr_with_empty_row_middle"])
def test_from_inserts_golden(golden, name):
    g = golden[name]
    r, c, v = from_data_inserts(g["rows"])
    m = Csr.from_inserts((len(g["rows"]), len(g["rows"][0])), r, c, v)
    assert m == Csr.from_data(g["rows"])
    assert np.asarray(m.row_index).tolist() == g["row_index"]


def random_stream(rng, n, rows, cols, dtype, zero_frac=0.1):
    r = rng.integers(0, rows, n).astype(np.uint64)
    r[: n // 2] = np.sort(r[: n // 2])  # a sorted prefix, then random order
    c = rng.integers(0, cols, n).astype(np.uint64)
    if np.dtype(dtype).kind == "f":
        v = rng.uniform(-2, 2, n).astype(dtype)
        z = rng.random(n) < zero_frac
        v[z] = np.where(rng.random(int(z.sum())) < 0.5, 0.0, -0.0).astype(dtype)
        v[rng.random(n) < 0.01] = np.nan  # NaN != default: kept
    else:
        v = rng.integers(0, 5, n).astype(dtype)
    return r, c, v


@pytest.mark.parametrize("dtype", [np.float64, np.float32, np.int32, np.uint32, np.int64, np.uint64])
@pytest.mark.parametrize("n,rows,cols", [(0, 5, 5), (1, 1, 1), (700, 50, 30), (200_000, 3000, 1000)])
def test_from_inserts_vs_oracle(orc, dtype, n, rows, cols):
    rng = np.random.default_rng(n + rows)
    r, c, v = random_stream(rng, n, rows, cols, dtype)
    m = Csr.from_inserts((rows, cols), r, c, v)
    assert_csr_bits(m, *orc.csr_from_inserts(rows, r, c, v))


def test_from_inserts_panics():
    r = np.array([0, 3], dtype=np.uint64)
    c = np.array([0, 0], dtype=np.uint64)
    with pytest.raises(Panic, match="big eek"):
        Csr.from_inserts((3, 3), r, c, np.array([1, 1], dtype=np.int32))
    m = Csr.from_inserts((3, 3), r, c, np.array([1, 0], dtype=np.int32))  # zero: skipped, no row extension
    assert np.asarray(m.row_index).tolist() == [0, 1, 1, 1]
    with pytest.raises(Panic):
        Csr.from_inserts((3, 3), np.array([0], dtype=np.uint64), np.array([3], dtype=np.uint64),
                         np.array([1], dtype=np.int32))


def bench_x(seed, k, n, fill, dtype):
    """The bench's RHS (sparse_dense_mul.rs:23-29): Dense k x n of zeros, then
    `fill` writes of v % 255 at (col % k, row % n) -- later writes win."""
    rng = np.random.default_rng(seed)
    cols = [np.zeros(n, dtype=dtype) for _ in range(k)]
    for _ in range(fill):
        j, i, v = int(rng.integers(0, k)), int(rng.integers(0, n)), rng.integers(0, 255)
        cols[j][i] = v
    return cols


@pytest.mark.parametrize("e", [10_000, 100_000, 900_000])
def test_bench_shape_u32_mul_dense_vs_oracle(orc, e):
    """sd_mul (sparse_dense_mul.rs:8-35) at e inserts: 1000 x 1000 u32, X of
    10 columns with e/100 random entries; wrapping u32 sums."""
    r, c, v = orc.gen_insert_stream(1000, e)
    a = Csr.from_inserts((1000, 1000), r, c, v.astype(np.uint32))
    x_cols = bench_x(1000 + e, 10, 1000, e // 100, np.uint32)
    got = a.mul_dense(Dense.from_columns(x_cols))
    rp, ci, vv = a.row_index, a.col_index, a.v
    assert_csr_bits(got, *orc.mul_dense(1000, 1000, rp, ci, vv, x_cols))
    assert np.diff(np.asarray(rp, np.int64)).max() > 8192 or e < 100_000  # the split kernel ran


@pytest.mark.parametrize("dtype", [np.int32, np.uint32, np.int64, np.uint64])
@pytest.mark.parametrize("k", [2, 7, 32, 70])
def test_split_spmm_forced_vs_oracle(orc, monkeypatch, dtype, k):
    """The nnz-balanced integer kernel on ordinary (unskewed) rows, forced by
    BSM_SPMM_SPLIT=1: rows that straddle chunks take the atomic path."""
    monkeypatch.setenv("BSM_SPMM_SPLIT", "1")
    rng = np.random.default_rng(k)
    rows, cols = 3000, 500
    lens = rng.integers(0, 3000, rows)
    lens[rng.random(rows) < 0.3] = 0
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    nnz = int(rp[-1])
    ci = rng.integers(0, cols, nnz).astype(np.uint64)
    v = rng.integers(-9, 10, nnz).astype(dtype) if np.dtype(dtype).kind == "i" else \
        rng.integers(0, 2**31, nnz).astype(dtype)
    a = Csr.from_csr_arrays((rows, cols), rp, ci, v)
    x_cols = [rng.integers(0, 1000, cols).astype(dtype) for _ in range(k)]
    got = a.mul_dense(Dense.from_columns(x_cols))
    assert_csr_bits(got, *orc.mul_dense(rows, cols, rp, ci, v, x_cols))


def test_skewed_f64_in_order_vs_oracle(orc):
    """A float matrix with one 150k-entry row keeps the in-order row kernel
    (float sums are not associative): bit-exact against the oracle."""
    r, c, v = orc.gen_insert_stream(77, 150_000, rows=500, cols=2000, vmod=1000)
    vals = (v.astype(np.float64) - 500.0) / 7.0
    a = Csr.from_inserts((500, 2000), r, c, vals)
    rng = np.random.default_rng(3)
    x_cols = [rng.uniform(-1, 1, 2000) for _ in range(5)]
    got = a.mul_dense(Dense.from_columns(x_cols))
    assert_csr_bits(got, *orc.mul_dense(500, 2000, a.row_index, a.col_index, a.v, x_cols))


# ---- From<COO<T>> for Csr<T> (sparse.rs:56-66) ------------------------------
def test_coo_to_csr_golden(golden):
    from basic_sparse_matrix_amd import COO

    g = golden["coo_to_csr"]  # sparse.rs:1443-1468
    coo = COO.with_capacity(tuple(g["dims"]), g["capacity"])
    for r, c, v in g["inserts"]:
        coo.insert((r, c, v))
    assert Csr.from_coo(coo) == Csr.from_data(g["rows"])


def test_coo_insert_out_of_bounds():
    from basic_sparse_matrix_amd import COO, MatErr, MatErrKind

    coo = COO.with_capacity((2, 3), 4)
    coo.insert((1, 2, 1.0))
    for bad in [(2, 0, 1.0), (0, 3, 1.0)]:
        with pytest.raises(MatErr) as e:
            coo.insert(bad)
        assert e.value.kind == MatErrKind.OutOfBounds


@pytest.mark.parametrize("dtype", [np.float64, np.float32, np.int32, np.uint64])
@pytest.mark.parametrize("n,rows,cols", [(0, 4, 4), (1, 1, 1), (5000, 300, 70), (400_000, 20_000, 5_000)])
def test_coo_to_csr_vs_oracle(orc, dtype, n, rows, cols):
    """Random entry order with many duplicate (row, col) keys: the stable sort
    keeps their insert order bit for bit."""
    from basic_sparse_matrix_amd import COO

    rng = np.random.default_rng(n + cols)
    r = rng.integers(0, rows, n).astype(np.uint64)
    c = rng.integers(0, max(1, cols // 3), n).astype(np.uint64)  # duplicates
    v = rng.integers(-4, 5, n).astype(dtype)
    coo = COO.with_capacity((rows, cols), n, dtype=dtype)
    for a, b, x in zip(r.tolist(), c.tolist(), v):
        coo.insert((a, b, x))
    got = Csr.from_coo(coo)
    assert_csr_bits(got, *orc.csr_from_coo(rows, cols, r, c, v))
