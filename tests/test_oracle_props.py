"""CPU-only checks of the oracle's internal consistency and of the
synthetic generator (no GPU): the band Cholesky restatement equals the
literal O(N^3) loop nest bit for bit; generated rows are sorted, distinct
and in range; mul_vector equals mul_dense with k = 1 on the reference's
own semantics where they coincide."""

import numpy as np
import pytest


def random_spd(rng, n, density, dtype):
    a = np.zeros((n, n))
    mask = rng.random((n, n)) < density
    a[mask] = rng.uniform(-1.0, 1.0, (n, n))[mask]
    a = np.tril(a, -1)
    a = a + a.T
    a[np.arange(n), np.arange(n)] = np.abs(a).sum(axis=1) + 1.0 + rng.random(n)
    return a.astype(dtype)


def csr_arrays(dense):
    nzr, nzc = np.nonzero(dense != 0)
    counts = np.bincount(nzr, minlength=dense.shape[0])
    return np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64), nzc.astype(np.uint64), dense[nzr, nzc]


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
@pytest.mark.parametrize("n,density", [(5, 0.6), (60, 0.1), (200, 0.03)])
def test_band_equals_literal_cholesky(orc, dtype, n, density):
    a = random_spd(np.random.default_rng(n), n, density, dtype)
    rp, ci, v = csr_arrays(a)
    lit = orc.cholesky(n, n, rp, ci, v, band=False)
    band = orc.cholesky(n, n, rp, ci, v, band=True)
    for x, y in zip(lit, band):
        assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_band_equals_literal_poisson(orc, dtype):
    g = 12
    rp, ci, v = orc.poisson2d(g)
    v = v.astype(dtype)
    n = g * g
    lit = orc.cholesky(n, n, rp, ci, v, band=False)
    band = orc.cholesky(n, n, rp, ci, v, band=True)
    for x, y in zip(lit, band):
        assert np.array_equal(np.asarray(x).view(np.uint8), np.asarray(y).view(np.uint8))
    b = orc.gen_x_cols(1002, n, 1, dtype=dtype)
    xs = [orc.solve(n, rp, ci, v, b, band=bb)[0] for bb in (False, True)]
    assert np.array_equal(xs[0].view(np.uint8), xs[1].view(np.uint8))


def test_poisson_structure(orc):
    rp, ci, v = orc.poisson2d(4)
    assert int(rp[-1]) == 5 * 16 - 4 * 4  # 5n - 4g
    assert list(ci[int(rp[5]):int(rp[6])]) == [1, 4, 5, 6, 9]
    assert list(v[int(rp[5]):int(rp[6])]) == [-1, -1, 4, -1, -1]


@pytest.mark.parametrize("kind,a,b", [(0, 10, 10), (1, 0, 60), (1, 990, 1000)])
def test_generator_rows_sorted_distinct(orc, kind, a, b):
    n_cols = 1000
    rp, ci, v = orc.gen_csr(1000, 500, n_cols, kind, a, b)
    for r in range(500):
        row = ci[int(rp[r]):int(rp[r + 1])].astype(np.int64)
        assert np.all(np.diff(row) > 0) and (row.size == 0 or (row[0] >= 0 and row[-1] < n_cols))
    assert np.all((v >= 0.5) & (v < 1.5))


def test_generator_deterministic(orc):
    a = orc.gen_csr(7, 100, 5000, 1, 0, 30)
    b = orc.gen_csr(7, 100, 5000, 1, 0, 30)
    c = orc.gen_csr(8, 100, 5000, 1, 0, 30)
    assert all(np.array_equal(x, y) for x, y in zip(a, b))
    assert not np.array_equal(a[1], c[1])


def test_mul_vector_matches_mul_dense_k1_on_sorted_rows(orc):
    rp, ci, v = orc.gen_csr(3, 300, 400, 1, 1, 20)
    x = orc.gen_x_cols(4, 400, 1)
    orp, oci, ov = orc.mul_dense(300, 400, rp, ci, v, x)
    out = orc.mul_vector(300, 400, rp, ci, v, x[0])
    dense = np.zeros(300)
    rows = np.repeat(np.arange(300), np.diff(orp.astype(np.int64)))
    dense[rows] = ov
    assert np.array_equal(out, dense)  # positive inputs: no dropped zeros, no -0


def test_u32_wrapping(orc):
    rp = np.array([0, 2], dtype=np.uint64)
    ci = np.array([0, 1], dtype=np.uint64)
    v = np.array([4_000_000_000, 3], dtype=np.uint32)
    x = [np.array([3, 5], dtype=np.uint32)]
    _, _, ov = orc.mul_dense(1, 2, rp, ci, v, x)
    assert int(ov[0]) == (4_000_000_000 * 3 + 15) % 2**32
