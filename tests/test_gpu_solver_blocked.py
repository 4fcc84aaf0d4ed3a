"""GPU tests of solve(..., order="blocked") (bsm_solve_blocked): the
reference's solve (src/lib.rs:11-24) with the triangular solves reassociated
into 64-row blocks. Not bit-exact by design; the bar is BASELINE.json's
floating-point tolerance: 1e-6 relative on f64 against the reference-order
result (the band oracle, itself pinned to the reference's goldens). The tests
use tighter bounds where the systems are well conditioned, so a wrong block
(an off-by-one in the band masks, a missing far block) cannot hide."""

import numpy as np
import pytest

from basic_sparse_matrix_amd import Csr, Dense, Panic, solve
from golden.golden_io import matrix, scalars

pytestmark = pytest.mark.gpu

TOL = {np.float64: 1e-10, np.float32: 2e-3}


def rel_err(x, ref):
    x = np.asarray(x, np.float64)
    ref = np.asarray(ref, np.float64)
    return np.linalg.norm(x - ref) / max(np.linalg.norm(ref), 1e-300)


def test_blocked_solve_golden(golden):
    """solve_test (lib.rs:74-138): [0.625, -0.1, 2.6999998, 0.5] within f32 rounding."""
    g = golden["solve_test"]
    b = Dense.from_data([scalars(c, np.float32) for c in g["b_cols"]], dtype=np.float32)
    a = Csr.from_data(matrix(g["rows"], np.float32), dtype=np.float32)
    x = solve(a, b, order="blocked").get_col(0)
    assert np.allclose(x, [0.625, -0.1, 2.6999998, 0.5], rtol=1e-6, atol=1e-6)


def test_blocked_solve_non_square_panics():
    with pytest.raises(Panic):
        solve(Csr.from_data([[1.0, 2.0]], dtype=np.float32), Dense.from_data([[1.0]], dtype=np.float32),
              order="blocked")


def test_blocked_solve_bad_order():
    with pytest.raises(ValueError):
        solve(Csr.from_data([[1.0]], dtype=np.float64), Dense.from_data([[1.0]], dtype=np.float64), order="x")


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("g,k", [(1, 1), (5, 2), (8, 1), (11, 3), (40, 2), (70, 1), (130, 2)])
def test_blocked_poisson_vs_oracle(orc, dtype, g, k):
    """2D Poisson g x g (bandwidth g): n from 1 to 16,900, one to three RHS
    columns; n not a multiple of 64 and bandwidths below, at and above the
    block size, so partial last blocks, empty far ranges and far blocks that
    straddle the band edge all occur."""
    n = g * g
    rp, ci, v = orc.poisson2d(g)
    v = v.astype(dtype)
    A = Csr.from_csr_arrays((n, n), rp, ci, v)
    b = orc.gen_x_cols(1004, n, k, dtype=dtype)
    ex = orc.solve(n, rp, ci, v, b, band=True)
    x = solve(A, Dense.from_columns(b), order="blocked")
    if dtype == np.float64:
        for j in range(k):
            assert rel_err(x.get_col(j), ex[j]) < TOL[dtype], j
    else:  # f32: error ~ cond(A) * 6e-8 (cond <= ~1e4 here) against the f64 solution
        x64 = orc.solve(n, rp, ci, v.astype(np.float64), [c.astype(np.float64) for c in b], band=True)
        for j in range(k):
            assert rel_err(x.get_col(j), x64[j]) < 2e-3, j


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_blocked_wide_band_vs_oracle(orc, dtype):
    """Bandwidth 1060 > 1024 (17 far blocks per 64-row block)."""
    n, g = 2400, 1060
    rows, cols, vals = [], [], []
    for i in range(n):
        for j, val in ((i - g, -1.0), (i - 1, -1.0), (i, 4.5), (i + 1, -1.0), (i + g, -1.0)):
            if 0 <= j < n:
                rows.append(i), cols.append(j), vals.append(val)
    rp = np.concatenate([[0], np.cumsum(np.bincount(rows, minlength=n))]).astype(np.uint64)
    ci = np.asarray(cols, dtype=np.uint64)
    v = np.asarray(vals, dtype=dtype)
    A = Csr.from_csr_arrays((n, n), rp, ci, v)
    b = orc.gen_x_cols(1003, n, 1, dtype=dtype)
    x = solve(A, Dense.from_columns(b), order="blocked").get_col(0)
    ex = orc.solve(n, rp, ci, v, b, band=True)[0]
    assert rel_err(x, ex) < TOL[dtype]


def test_blocked_random_spd_vs_oracle(orc):
    """Random sparse SPD (irregular envelope, dense-ish rows) against the
    literal oracle."""
    rng = np.random.default_rng(7)
    n = 300
    a = np.zeros((n, n))
    mask = rng.random((n, n)) < 0.02
    vals = rng.uniform(-1.0, 1.0, (n, n))
    a[mask] = vals[mask]
    a = np.tril(a, -1)
    a = a + a.T
    a[np.arange(n), np.arange(n)] = np.abs(a).sum(axis=1) + 1.0 + rng.random(n)
    nzr, nzc = np.nonzero(a != 0)
    rp = np.concatenate([[0], np.cumsum(np.bincount(nzr, minlength=n))]).astype(np.uint64)
    ci, v = nzc.astype(np.uint64), a[nzr, nzc]
    A = Csr.from_csr_arrays((n, n), rp, ci, v)
    b = orc.gen_x_cols(1005, n, 2)
    ex = orc.solve(n, rp, ci, v, b, band=False)
    x = solve(A, Dense.from_columns(b), order="blocked")
    for j in range(2):
        assert rel_err(x.get_col(j), ex[j]) < 1e-12


# the blocked factor (blk_chol) / the reference-order band factor (band_chol5)
# under the blocked solves (BSM_BLK_CHOL=0)
@pytest.mark.parametrize("blk_chol", ["1", "0"])
def test_blocked_poisson_250_f64_vs_reference_order(orc, monkeypatch, blk_chol):
    """62,500 unknowns, bandwidth 250: blocked vs reference order on the GPU."""
    monkeypatch.setenv("BSM_BLK_CHOL", blk_chol)
    g = 250
    n = g * g
    rp, ci, v = orc.poisson2d(g)
    A = Csr.from_csr_arrays((n, n), rp, ci, v)
    b = orc.gen_x_cols(1002, n, 1)
    xr = solve(A, Dense.from_columns(b)).get_col(0)
    xb = solve(A, Dense.from_columns(b), order="blocked").get_col(0)
    assert rel_err(xb, xr) < 1e-10


@pytest.mark.slow
def test_c5_blocked_poisson_1m_f64_properties(orc, golden_c5):
    """C5 (N = 1M, bandwidth 1000) through the blocked solves: within 1e-6
    relative (BASELINE.json) of the band oracle's exact x (sampled from
    tests/golden/c5_poisson_1000.json) and of x_true, residual tiny."""
    g = 1000
    n = g * g
    rp, ci, v = orc.poisson2d(g)
    A = Csr.from_csr_arrays((n, n), rp, ci, v)
    x_true = orc.gen_x_cols(1002, n, 1)[0]
    rows = np.repeat(np.arange(n), np.diff(rp.astype(np.int64)))
    b = np.zeros(n)
    np.add.at(b, rows, v * x_true[ci.astype(np.int64)])
    x = solve(A, Dense.from_columns([b]), order="blocked").get_col(0)
    exact = np.asarray([int(h, 16) for h in golden_c5["x_sample_bits"]], dtype=np.uint64).view(np.float64)
    assert rel_err(x[::golden_c5["x_stride"]], exact) < 1e-6
    assert rel_err(x, x_true) < 1e-6
    r = np.zeros(n)
    np.add.at(r, rows, v * x[ci.astype(np.int64)])
    assert np.linalg.norm(r - b) / np.linalg.norm(b) < 1e-12


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("g,k", [(9, 1), (40, 2), (70, 1), (130, 2), (250, 1)])
def test_blocked_progressive_handoff_deterministic(orc, dtype, g, k):
    """The blocked factor's progressive hand-off (tile K publishes Linv_K by
    16-row blocks, tile K + 1 forms its sub-diagonal tile block by block):
    two runs give the same bits (every element's MFMA sequence is fixed, so
    any stale hand-off would show), within the tolerance of the band oracle."""
    n = g * g
    rp, ci, v = orc.poisson2d(g)
    v = v.astype(dtype)
    A = Csr.from_csr_arrays((n, n), rp, ci, v)
    b = orc.gen_x_cols(1007, n, k, dtype=dtype)
    xs = []
    for _ in range(2):
        x = solve(A, Dense.from_columns(b), order="blocked")
        xs.append([np.asarray(x.get_col(j)).copy() for j in range(k)])
    ref = orc.solve(n, rp, ci, v.astype(np.float64), [c.astype(np.float64) for c in b], band=True)
    for j in range(k):
        assert np.array_equal(xs[0][j].view(np.uint8), xs[1][j].view(np.uint8)), j
        assert rel_err(xs[0][j], ref[j]) < TOL[dtype], j
