"""GPU parity of the general exact Cholesky path (kernels_solve.hip
`chol_general`): the inputs the band kernels refuse, with the reference's
semantics (src/sparse.rs:682-714, get_row_complete :267-294, solve
lib.rs:11-65):

* non-positive or non-finite pivots: powf(0.5) of a negative stores NaN,
  1/0 gives inf, and the loop carries on (every later L[i][j] turns NaN);
* rows with unsorted or duplicate columns, read through get_row_complete's
  shifted vector;
* `l.get_row_complete(j).unwrap()` on a row no insert has registered yet
  (sparse.rs:707) -> Panic;
* bands wider than the band kernels take.

Bar: bit-exact against the literal oracle (oracle/bsm_oracle_tpl.inc
orc_cholesky_literal_, orc_solve_ with use_band=0); NaN compares equal to
NaN whatever its payload (the reference's NaN bits are its host's).
"""

import numpy as np
import pytest

from basic_sparse_matrix_amd import Csr, Dense, Panic, solve

pytestmark = pytest.mark.gpu


def same_bits(a, b):
    """Bit-equal, except that any NaN equals any NaN."""
    a, b = np.asarray(a), np.asarray(b)
    if a.shape != b.shape or a.dtype != b.dtype:
        return False
    na, nb = np.isnan(a), np.isnan(b)
    if not np.array_equal(na, nb):
        return False
    u = np.uint64 if a.dtype.itemsize == 8 else np.uint32
    return np.array_equal(a[~na].view(u), b[~nb].view(u))


def assert_l_matches(got: Csr, rp, ci, v):
    assert np.array_equal(np.asarray(got.row_index, np.uint64), np.asarray(rp, np.uint64))
    assert np.array_equal(np.asarray(got.col_index, np.uint64), np.asarray(ci, np.uint64))
    assert same_bits(got.v, np.asarray(v, dtype=got.dtype))


def csr_arrays(dense):
    nzr, nzc = np.nonzero(dense != 0)
    counts = np.bincount(nzr, minlength=dense.shape[0])
    rp = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
    return rp, nzc.astype(np.uint64), dense[nzr, nzc]


def random_sym(rng, n, density, dtype, diag):
    a = np.zeros((n, n))
    mask = rng.random((n, n)) < density
    a[mask] = rng.uniform(-1.0, 1.0, (n, n))[mask]
    a = np.tril(a, -1)
    a = a + a.T
    a[np.arange(n), np.arange(n)] = diag
    return a.astype(dtype)


def check_chol_and_solve(orc, A: Csr, rp, ci, v, n, dtype, k=2, seed=5):
    L = A.cholesky_decomp()
    assert_l_matches(L, *orc.cholesky(n, n, rp, ci, v, band=False))
    b = [np.random.default_rng(seed + j).uniform(-1, 1, n).astype(dtype) for j in range(k)]
    check_solve(orc, A, rp, ci, v, n, b)


def check_solve(orc, A, rp, ci, v, n, b):
    """x bit-equal to the oracle's; where the reference panics (an empty row
    of L or L*: `row.last().unwrap()` / `row[0]`, lib.rs:41, :60), so does
    the GPU."""
    try:
        ex = orc.solve(n, rp, ci, v, b, band=False)
    except orc.OracleError:
        with pytest.raises(Panic):
            solve(A, Dense.from_columns(b))
        return
    x = solve(A, Dense.from_columns(b))
    for j in range(len(b)):
        assert same_bits(x.get_col(j), ex[j])


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("n,density", [(1, 1.0), (9, 0.4), (70, 0.1), (257, 0.03)])
def test_forced_general_equals_literal_on_spd(orc, monkeypatch, dtype, n, density):
    """BSM_CHOL_GENERAL=1 runs the general path on SPD inputs: the same bits
    as the literal oracle (and so as the band kernels)."""
    monkeypatch.setenv("BSM_CHOL_GENERAL", "1")
    rng = np.random.default_rng(n + 11)
    a = random_sym(rng, n, density, dtype, 0.0)
    a[np.arange(n), np.arange(n)] = np.abs(a).sum(axis=1) + 1.0 + rng.random(n)
    rp, ci, v = csr_arrays(a)
    check_chol_and_solve(orc, Csr.from_csr_arrays((n, n), rp, ci, v), rp, ci, v, n, dtype)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("n,seed", [(6, 1), (40, 2), (130, 3)])
def test_indefinite_matrix_stores_nan(orc, dtype, n, seed):
    """A symmetric indefinite matrix: some pivot's radicand is negative,
    powf(0.5) gives NaN and every later entry is NaN, as in the reference."""
    rng = np.random.default_rng(seed)
    a = random_sym(rng, n, 0.3, dtype, rng.uniform(-0.5, 1.0, n))
    rp, ci, v = csr_arrays(a)
    L = Csr.from_csr_arrays((n, n), rp, ci, v).cholesky_decomp()
    assert np.isnan(np.asarray(L.v)).any()  # the case is really exercised
    check_chol_and_solve(orc, Csr.from_csr_arrays((n, n), rp, ci, v), rp, ci, v, n, dtype)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_zero_pivot_gives_inf_and_nan(orc, dtype):
    """A[1][1] = A[1][0]^2 / A[0][0] exactly: pivot 1 is +0, so column 1 is
    1/0 * temp = +-inf (temp != 0) or NaN (temp == 0)."""
    a = np.array([[4.0, 2.0, 0.0, 1.0],
                  [2.0, 1.0, 3.0, 0.0],
                  [0.0, 3.0, 5.0, 0.0],
                  [1.0, 0.0, 0.0, 2.0]], dtype=dtype)
    rp, ci, v = csr_arrays(a)
    L = Csr.from_csr_arrays((4, 4), rp, ci, v).cholesky_decomp()
    assert np.isinf(np.asarray(L.v)).any()
    check_chol_and_solve(orc, Csr.from_csr_arrays((4, 4), rp, ci, v), rp, ci, v, 4, dtype)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("n,seed", [(5, 7), (50, 8), (200, 9)])
def test_unsorted_and_duplicate_rows(orc, dtype, n, seed):
    """Rows stored out of column order (insert in any order, sparse.rs:222-250)
    and with a repeated column: get_row_complete shifts the row, and the
    factor reads the shifted positions."""
    rng = np.random.default_rng(seed)
    a = random_sym(rng, n, 0.2, dtype, 0.0)
    a[np.arange(n), np.arange(n)] = np.abs(a).sum(axis=1) + 2.0
    rp, ci, v = csr_arrays(a)
    ci2, v2 = ci.copy(), v.copy()
    for i in range(n):  # reverse every third row, duplicate a column in every fifth
        s, e = int(rp[i]), int(rp[i + 1])
        if i % 3 == 0:
            ci2[s:e] = ci2[s:e][::-1]
            v2[s:e] = v2[s:e][::-1]
        elif i % 5 == 1 and e - s >= 2:
            ci2[s + 1] = ci2[s]
    A = Csr.from_csr_arrays((n, n), rp, ci2, v2)
    L = A.cholesky_decomp()
    assert_l_matches(L, *orc.cholesky(n, n, rp, ci2, v2, band=False))
    check_solve(orc, A, rp, ci2, v2, n, [np.linspace(-1, 1, n).astype(dtype)])


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_unsorted_upper_entries_solve(orc, dtype):
    """Rows whose entries past the diagonal are stored out of order: the
    shift lands only on positions the factor never reads (j <= i), so L is
    finite and the whole solve is compared, not just the panic."""
    n = 300
    rng = np.random.default_rng(12)
    a = random_sym(rng, n, 0.05, dtype, 0.0)
    a[np.arange(n), np.arange(n)] = np.abs(a).sum(axis=1) + 1.0
    rp, ci, v = csr_arrays(a)
    ci2, v2 = ci.copy(), v.copy()
    swapped = 0
    for i in range(n):
        s, e = int(rp[i]), int(rp[i + 1])
        if e - s >= 3 and ci2[e - 2] > i:
            ci2[e - 2], ci2[e - 1] = ci2[e - 1], ci2[e - 2]
            v2[e - 2], v2[e - 1] = v2[e - 1], v2[e - 2]
            swapped += 1
    assert swapped > 10
    A = Csr.from_csr_arrays((n, n), rp, ci2, v2)
    L = A.cholesky_decomp()
    assert not np.isnan(np.asarray(L.v)).any()
    assert_l_matches(L, *orc.cholesky(n, n, rp, ci2, v2, band=False))
    b = [np.linspace(-1, 1, n).astype(dtype), np.cos(np.arange(n)).astype(dtype)]
    x = solve(A, Dense.from_columns(b))
    ex = orc.solve(n, rp, ci2, v2, b, band=False)
    for j in range(2):
        assert same_bits(x.get_col(j), ex[j])


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_unregistered_row_unwrap_panics(orc, dtype):
    """Row 1 of L is all zero (pivot 0, nothing stored) and row 2 has nothing
    before column 1: `l.get_row_complete(1).unwrap()` is None (sparse.rs:707)."""
    a = np.array([[1.0, 0.0, 0.0], [0.0, 0.0, 0.0], [0.0, 0.0, 1.0]], dtype=dtype)
    rp, ci, v = csr_arrays(a)
    with pytest.raises(orc.OracleError):
        orc.cholesky(3, 3, rp, ci, v, band=False)
    with pytest.raises(Panic):
        Csr.from_csr_arrays((3, 3), rp, ci, v).cholesky_decomp()


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_band_wider_than_band_kernels(orc, dtype):
    """One far entry (A[n-1][0]) makes the band n-1 = 1199 > the band kernels'
    1073: the general path factors it, bit-exact."""
    n = 1200
    a = np.zeros((n, n), dtype=dtype)
    i = np.arange(n)
    a[i, i] = 4.0
    a[i[1:], i[1:] - 1] = a[i[:-1], i[:-1] + 1] = -1.0
    a[n - 1, 0] = a[0, n - 1] = 0.5
    rp, ci, v = csr_arrays(a)
    check_chol_and_solve(orc, Csr.from_csr_arrays((n, n), rp, ci, v), rp, ci, v, n, dtype, k=1)


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_forward_substitution_nonfinite_entry_past_diagonal(orc, dtype):
    """forward_substitution adds e.v * y[e.col] for every entry off the
    diagonal (lib.rs:36-39); past the diagonal y is still 0, so an inf entry
    there contributes NaN and y[row] is NaN -- finite ones contribute +-0."""
    from basic_sparse_matrix_amd import forward_substitution
    rows = np.array([[2.0, 0.0, 5.0, 0.0],
                     [1.0, 3.0, 0.0, np.inf],
                     [0.0, 1.0, 4.0, 0.0],
                     [1.0, 0.0, 2.0, 1.0]], dtype=dtype)
    rp, ci, v = csr_arrays(rows)
    L = Csr.from_csr_arrays((4, 4), rp, ci, v)
    b = [np.array([1.0, 2.0, 3.0, 4.0], dtype=dtype)]
    y = forward_substitution(L, Dense.from_columns(b))
    ex = orc.forward_substitution(4, rp, ci, v, b)
    assert np.isnan(ex[0][1])
    assert same_bits(y.get_col(0), ex[0])
