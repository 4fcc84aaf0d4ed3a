"""GPU parity of the sparse x sparse operations:
Csr::add_sparse / sub_sparse (src/sparse.rs:484-599) and Csr::mul_sparse
(src/sparse.rs:601-635), against the reference's unit tests and the CPU
oracle's literal restatement (oracle/, pinned in test_oracle_golden.py).
Inputs include the reference benches' shapes (benches/sparse_dense_mul.rs
ss_add, benches/sparse_sparse_mul.rs ss_mul: random insert order, so rows
with unsorted and repeated columns), where the merge semantics matter.
The bar is bit-exact.
"""

import numpy as np
import pytest

from basic_sparse_matrix_amd import Csr, MatErr, MatErrKind, Panic
from test_gpu_spmm import assert_csr_bits

pytestmark = pytest.mark.gpu


def arrays(m: Csr):
    return (m.dims.rows, m.dims.cols, np.asarray(m.row_index, np.uint64), np.asarray(m.col_index, np.uint64),
            np.asarray(m.v))


def test_add_sub_golden(golden):
    for name, op in [("add_sparse", Csr.add_sparse), ("sub_sparse", Csr.sub_sparse)]:
        g = golden[name]
        assert op(Csr.from_data(g["a"]), Csr.from_data(g["b"])) == Csr.from_data(g["c"]), name


def test_mul_sparse_golden(golden):
    g = golden["sparse_multiplication"]
    a = Csr.from_data(g["a"])
    assert a.mul_sparse(a.transpose()) == Csr.from_data(g["c"])


def test_errors():
    a = Csr.from_data([[1, 2]])
    with pytest.raises(MatErr) as e:
        a.add_sparse(Csr.from_data([[1], [2]]))
    assert e.value.kind == MatErrKind.IncorrectDimensions
    with pytest.raises(MatErr):
        a.sub_sparse(Csr.from_data([[1], [2]]))
    with pytest.raises(Panic, match="big eek"):  # a 0-row Csr cannot even be finalised (sparse.rs:209-211)
        Csr.new((0, 3)).finalise()
    # mul_sparse has no dimension check: a (1 x 2) times a (1 x 2)
    out = a.mul_sparse(Csr.from_data([[3, 4]]))
    assert out.get_dims().rows == 1 and out.get_dims().cols == 2


def sorted_random(rng, rows, cols, density, dtype):
    if np.dtype(dtype).kind == "f":
        d = rng.uniform(-2, 2, (rows, cols)).astype(dtype)
    else:
        d = rng.integers(1, 9, (rows, cols)).astype(dtype)
    d[rng.random((rows, cols)) >= density] = 0
    return Csr.from_data(d.tolist(), dtype=dtype)


def unsorted_random(rng, e, rows, cols, dtype, seed_shift=0):
    """Bench-shaped: e inserts in random (row, col) order -> running-max rows,
    unsorted and repeated columns inside rows (sparse.rs:237-250)."""
    r = rng.integers(0, rows, e).astype(np.uint64)
    c = rng.integers(0, cols, e).astype(np.uint64)
    if np.dtype(dtype).kind == "f":
        v = rng.uniform(-3, 3, e).astype(dtype)
    else:
        v = rng.integers(0, 255, e).astype(dtype)
    return Csr.from_inserts((rows, cols), r, c, v)


DTYPES = [np.float64, np.float32, np.int32, np.uint32, np.int64, np.uint64]


@pytest.mark.parametrize("path", ["wave", "general"])
@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("kind", ["sorted", "unsorted"])
def test_add_sub_vs_oracle(orc, monkeypatch, dtype, kind, path):
    """Both add/sub paths: one wave per row when every row fits one wave's
    LDS (addsub_wave, the default for such operands), and the general
    count / long-row / piece pipeline (BSM_SS_WAVE=0)."""
    if path == "general":
        monkeypatch.setenv("BSM_SS_WAVE", "0")
    rng = np.random.default_rng(11)
    if kind == "sorted":
        a, b = sorted_random(rng, 120, 90, 0.1, dtype), sorted_random(rng, 120, 90, 0.1, dtype)
    else:
        a, b = unsorted_random(rng, 20_000, 300, 200, dtype), unsorted_random(rng, 20_000, 300, 200, dtype)
    assert_csr_bits(a.add_sparse(b), *orc.add_sparse(arrays(a), arrays(b)))
    assert_csr_bits(a.sub_sparse(b), *orc.sub_sparse(arrays(a), arrays(b)))
    assert_csr_bits(b.sub_sparse(a), *orc.sub_sparse(arrays(b), arrays(a)))


@pytest.mark.parametrize("path", ["wave", "general"])
@pytest.mark.parametrize("dtype", [np.float64, np.uint32, np.int64])
def test_add_sub_moderate_unsorted_rows(orc, monkeypatch, dtype, path):
    """Rows of 0 to 1,000 entries per side (the wave path's range, up to its
    2,048-entry cap together) with unsorted and repeated columns: the merge's
    every branch (greater, less, equal, one side exhausted) inside one wave's
    LDS, and rows with zero results dropped."""
    if path == "general":
        monkeypatch.setenv("BSM_SS_WAVE", "0")
    rng = np.random.default_rng(23)
    rows, cols = 400, 300

    def make():
        lens = rng.integers(0, 1001, rows)
        lens[:3] = [0, 1000, 1]
        rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
        ci = rng.integers(0, cols, int(rp[-1])).astype(np.uint64)
        if np.dtype(dtype).kind == "f":
            v = rng.integers(-2, 3, int(rp[-1])).astype(dtype)  # zeros and exact cancellations
        else:
            v = rng.integers(1, 4, int(rp[-1])).astype(dtype)
        return Csr.from_csr_arrays((rows, cols), rp, ci, v)

    a, b = make(), make()
    for op, ref in [(Csr.add_sparse, orc.add_sparse), (Csr.sub_sparse, orc.sub_sparse)]:
        assert_csr_bits(op(a, b), *ref(arrays(a), arrays(b)))
        assert_csr_bits(op(b, a), *ref(arrays(b), arrays(a)))


def test_sub_exact_cancellation(orc):
    """a - a: every stored value cancels exactly and is dropped (insert's zero
    skip); rhs-only entries are T::default() - v."""
    rng = np.random.default_rng(2)
    a = sorted_random(rng, 50, 40, 0.2, np.float64)
    z = a.sub_sparse(a)
    assert z.get_nnz() == 0 and np.asarray(z.row_index).tolist() == [0] * 51
    b = Csr.new((50, 40), dtype=np.float64).finalise()
    assert_csr_bits(b.sub_sparse(a), *orc.sub_sparse(arrays(b), arrays(a)))


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("shape", [(60, 45, 70), (200, 300, 150), (1, 1, 1)])
def test_mul_sparse_sorted_vs_oracle(orc, dtype, shape):
    rng = np.random.default_rng(sum(shape))
    m, k, n = shape
    a, b = sorted_random(rng, m, k, 0.08, dtype), sorted_random(rng, k, n, 0.08, dtype)
    assert_csr_bits(a.mul_sparse(b), *orc.mul_sparse(arrays(a), arrays(b)))


@pytest.mark.parametrize("dtype", [np.float64, np.uint32, np.int64])
@pytest.mark.parametrize("e", [1_000, 20_000, 100_000])
def test_mul_sparse_bench_shape_vs_oracle(orc, dtype, e):
    """ss_mul (sparse_sparse_mul.rs:6-37) shape at e inserts per operand:
    1000 x 1000, random insert order (unsorted, repeated columns)."""
    rng = np.random.default_rng(e)
    a = unsorted_random(rng, e, 1000, 1000, dtype)
    b = unsorted_random(rng, e, 1000, 1000, dtype)
    assert_csr_bits(a.mul_sparse(b), *orc.mul_sparse(arrays(a), arrays(b)))


def test_mul_sparse_rectangular_mismatch(orc):
    """No dimension check in the reference: a.cols != b.rows still merges."""
    rng = np.random.default_rng(9)
    a = sorted_random(rng, 30, 50, 0.2, np.int32)
    b = sorted_random(rng, 20, 40, 0.2, np.int32)
    assert_csr_bits(a.mul_sparse(b), *orc.mul_sparse(arrays(a), arrays(b)))


@pytest.mark.parametrize("case", ["both_have_max", "rhs_lacks_max", "unequal_max_counts", "one_side_empty",
                                  "sorted_long", "sorted_duplicates", "one_sorted", "all_equal",
                                  "descending_equal", "descending", "three_columns", "wide_columns"])
def test_add_sub_long_rows_vs_oracle(orc, case):
    """Rows above the piece threshold (64 entries) are cut at the pairs of
    the row maximum, then again inside each piece (at the piece's maximum, or
    by value when both sides are sorted); every way the maxima can be
    distributed stays exact, including inputs that defeat the cut (equal
    descending rows: the scan budget)."""
    rng = np.random.default_rng(len(case))
    n, cols = 30_000, 500
    ca = rng.integers(0, cols, n)
    cb = rng.integers(0, cols, n)
    if case == "rhs_lacks_max":
        cb = np.minimum(cb, cols - 2)
    if case == "unequal_max_counts":
        ca[rng.random(n) < 0.05] = cols - 1
    if case == "sorted_long":
        ca, cb = np.sort(ca), np.sort(cb)
    if case == "sorted_duplicates":
        ca, cb = np.sort(ca // 50), np.sort(cb[: n // 3] // 50)
    if case == "one_sorted":
        ca = np.sort(ca)
    if case == "all_equal":
        ca, cb = np.full(n, 7), np.full(n // 2, 7)
    if case == "descending_equal":
        ca = np.sort(ca)[::-1].copy()
        cb = ca.copy()
    if case == "descending":
        ca, cb = np.sort(ca)[::-1].copy(), np.sort(cb)[::-1].copy()
    if case == "three_columns":
        ca, cb = ca % 3, cb % 3
    if case == "wide_columns":
        cols = 1 << 30
        ca, cb = rng.integers(0, cols, n), rng.integers(0, cols, n)
    if case == "one_side_empty":
        cb = cb[:0]
    va = rng.integers(-3, 4, len(ca)).astype(np.int64)
    vb = rng.integers(-3, 4, len(cb)).astype(np.int64)
    va[va == 0] = 1
    vb[vb == 0] = 2
    a = Csr.from_csr_arrays((2, cols), np.array([0, 5, len(ca)], np.uint64), ca.astype(np.uint64), va)
    b = Csr.from_csr_arrays((2, cols), np.array([0, min(3, len(cb)), len(cb)], np.uint64), cb.astype(np.uint64), vb)
    for op, ref in [(Csr.add_sparse, orc.add_sparse), (Csr.sub_sparse, orc.sub_sparse)]:
        assert_csr_bits(op(a, b), *ref(arrays(a), arrays(b)))
        assert_csr_bits(op(b, a), *ref(arrays(b), arrays(a)))


@pytest.mark.parametrize("dtype", [np.uint32, np.float64])
@pytest.mark.parametrize("e", [300_000])
def test_add_sub_bench_shape_vs_oracle(orc, dtype, e):
    """ss_add (benches/sparse_dense_mul.rs:37-67) shape: 1000 x 1000, e random
    inserts per operand, so ~all entries pile into the last row (running-max
    rule) with unsorted, repeated columns; rows 990-998 hold hundreds."""
    rng = np.random.default_rng(e + 1)
    a = unsorted_random(rng, e, 1000, 1000, dtype)
    b = unsorted_random(rng, e, 1000, 1000, dtype)
    assert_csr_bits(a.add_sparse(b), *orc.add_sparse(arrays(a), arrays(b)))
    assert_csr_bits(a.sub_sparse(b), *orc.sub_sparse(arrays(a), arrays(b)))
