"""GPU tests of solve(..., order="nd") (bsm_solve_nd): x = A^-1 b
(src/lib.rs:11-24) by a multifrontal Cholesky of P A P^T, P a
nested-dissection order (csrc/nd_order.cpp, csrc/kernels_nd.hip). Another
elimination order, so not bit-exact; the bar is BASELINE.json's f64
tolerance, 1e-6 relative against the reference-order result (the band
oracle, pinned to the reference's goldens). Tighter bounds where the systems
are well conditioned, so a wrong front row, a missed child update or a stale
tile hand-off cannot hide. Leaf sizes from 1 to whole-matrix fronts cover
separator trees from deep and narrow to a single dense front."""

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


def csr_arrays(a):
    nzr, nzc = np.nonzero(a != 0)
    n = a.shape[0]
    rp = np.concatenate([[0], np.cumsum(np.bincount(nzr, minlength=n))]).astype(np.uint64)
    return rp, nzc.astype(np.uint64), a[nzr, nzc]


def residual(rp, ci, v, x, b):
    n = len(rp) - 1
    rows = np.repeat(np.arange(n), np.diff(rp.astype(np.int64)))
    r = np.zeros(n)
    np.add.at(r, rows, v.astype(np.float64) * np.asarray(x, np.float64)[ci.astype(np.int64)])
    return np.linalg.norm(r - b) / max(np.linalg.norm(b), 1e-300)


def test_nd_solve_golden(golden):
    """solve_test (lib.rs:74-138): [0.625, -0.1, 2.6999998, 0.5] within f32 rounding."""
    g = golden["solve_test"]
    b = Dense.from_data([scalars(c, np.float32) for c in g["b_cols"]], dtype=np.float32)
    a = Csr.from_data(matrix(g["rows"], np.float32), dtype=np.float32)
    x = solve(a, b, order="nd").get_col(0)
    assert np.allclose(x, [0.625, -0.1, 2.6999998, 0.5], rtol=1e-6, atol=1e-6)


def test_nd_solve_non_square_panics():
    with pytest.raises(Panic):
        solve(Csr.from_data([[1.0, 2.0]], dtype=np.float32), Dense.from_data([[1.0]], dtype=np.float32), order="nd")


def test_nd_not_positive_definite_raises():
    a = Csr.from_data([[1.0, 2.0], [2.0, 1.0]], dtype=np.float64)
    with pytest.raises(Exception, match="positive definite"):
        solve(a, Dense.from_columns([np.array([1.0, 1.0])]), order="nd")


@pytest.mark.parametrize("leaf", ["1", "8", "64", "256", "100000"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("g,k", [(1, 1), (5, 2), (11, 3), (40, 2), (70, 1), (130, 2)])
def test_nd_poisson_vs_oracle(orc, monkeypatch, dtype, g, k, leaf):
    """2D Poisson g x g, one to three RHS columns, leaf parts from single
    vertices (every node a 64-padded front of one pivot) to one dense front."""
    if leaf == "1" and g > 40:
        pytest.skip("leaf 1 at this size: thousands of one-pivot fronts, covered at g <= 40")
    if leaf == "100000" and g > 70:
        pytest.skip("one dense front of n > 4900: covered at g <= 70")
    monkeypatch.setenv("BSM_ND_LEAF", leaf)
    n = g * g
    rp, ci, v = orc.poisson2d(g)
    v = v.astype(dtype)
    A = Csr.from_csr_arrays((n, n), rp, ci, v)
    b = orc.gen_x_cols(1004, n, k, dtype=dtype)
    x = solve(A, Dense.from_columns(b), order="nd")
    if dtype == np.float64:
        ex = orc.solve(n, rp, ci, v, b, band=True)
        for j in range(k):
            assert rel_err(x.get_col(j), ex[j]) < TOL[dtype], j
    else:
        x64 = orc.solve(n, rp, ci, v.astype(np.float64), [c.astype(np.float64) for c in b], band=True)
        for j in range(k):
            assert rel_err(x.get_col(j), x64[j]) < 2e-3, j


def test_nd_random_spd_vs_oracle(orc):
    """Random sparse SPD (irregular graph) against the literal oracle."""
    rng = np.random.default_rng(7)
    n = 300
    a = np.zeros((n, n))
    mask = rng.random((n, n)) < 0.02
    vals = rng.uniform(-1.0, 1.0, (n, n))
    a[mask] = vals[mask]
    a = np.tril(a, -1)
    a = a + a.T
    a[np.arange(n), np.arange(n)] = np.abs(a).sum(axis=1) + 1.0 + rng.random(n)
    rp, ci, v = csr_arrays(a)
    A = Csr.from_csr_arrays((n, n), rp, ci, v)
    b = orc.gen_x_cols(1005, n, 2)
    ex = orc.solve(n, rp, ci, v, b, band=False)
    x = solve(A, Dense.from_columns(b), order="nd")
    for j in range(2):
        assert rel_err(x.get_col(j), ex[j]) < 1e-12


def test_nd_lower_triangle_only(orc):
    """cholesky_decomp reads A[i][j] for j <= i only: a matrix stored as its
    lower triangle solves as the full symmetric one."""
    g = 30
    n = g * g
    rp, ci, v = orc.poisson2d(g)
    rows = np.repeat(np.arange(n), np.diff(rp.astype(np.int64)))
    keep = ci.astype(np.int64) <= rows
    rpl = np.concatenate([[0], np.cumsum(np.bincount(rows[keep], minlength=n))]).astype(np.uint64)
    b = orc.gen_x_cols(1006, n, 1)
    x_full = solve(Csr.from_csr_arrays((n, n), rp, ci, v), Dense.from_columns(b), order="nd").get_col(0)
    x_low = solve(Csr.from_csr_arrays((n, n), rpl, ci[keep], v[keep]), Dense.from_columns(b), order="nd").get_col(0)
    assert np.array_equal(np.asarray(x_full), np.asarray(x_low))


def test_nd_disconnected_blocks(orc):
    """Block-diagonal: two grids and isolated vertices (separator-free splits,
    fronts without pivots that only pass updates through)."""
    import scipy.sparse as sp

    g = 12
    n1 = g * g
    rp, ci, v = orc.poisson2d(g)
    P = sp.csr_matrix((v, ci.astype(np.int64), rp.astype(np.int64)), shape=(n1, n1))
    M = sp.block_diag([P, 2.0 * P, sp.identity(9) * 3.0], format="csr")
    M.sort_indices()
    n = M.shape[0]
    rp2, ci2, v2 = M.indptr.astype(np.uint64), M.indices.astype(np.uint64), M.data.astype(np.float64)
    b = orc.gen_x_cols(1008, n, 1)
    x = solve(Csr.from_csr_arrays((n, n), rp2, ci2, v2), Dense.from_columns(b), order="nd").get_col(0)
    ex = orc.solve(n, rp2, ci2, v2, b, band=True)[0]
    assert rel_err(x, ex) < 1e-12


def test_nd_wide_irregular_graph_residual():
    """n = 20,000, random graph (bandwidth ~ n: beyond the band kernels and the
    general path's n <= 16,384): the nd order still factors it; checked by
    the residual (no oracle finishes this in seconds)."""
    import scipy.sparse as sp

    rng = np.random.default_rng(11)
    n, deg = 20000, 2
    r = rng.integers(0, n, n * deg)
    c = rng.integers(0, n, n * deg)
    m = sp.coo_matrix((rng.uniform(-1, 1, len(r)), (r, c)), shape=(n, n)).tocsr()
    m = m + m.T
    m = m + sp.diags(np.asarray(abs(m).sum(axis=1)).ravel() + 1.0)
    m = m.tocsr()
    m.sum_duplicates()
    m.sort_indices()
    rp, ci, v = m.indptr.astype(np.uint64), m.indices.astype(np.uint64), m.data.astype(np.float64)
    b = rng.uniform(-1, 1, n)
    x = solve(Csr.from_csr_arrays((n, n), rp, ci, v), Dense.from_columns([b]), order="nd").get_col(0)
    assert residual(rp, ci, v, x, b) < 1e-12


@pytest.mark.parametrize("g", [64, 250])
def test_nd_deterministic(orc, monkeypatch, g):
    """Fixed tile order, fixed child order in the extend-add and the solves,
    and an analysis whose result does not depend on its threads' timing: two
    fresh handles with no plan cache anywhere (BSM_ND_CACHE=0: the bisection,
    symbolic pass and layout run again for each) give the same bits, and so
    does a third solve through the cached plan."""
    n = g * g
    rp, ci, v = orc.poisson2d(g)
    b = orc.gen_x_cols(1007, n, 1)
    monkeypatch.setenv("BSM_ND_CACHE", "0")
    x0 = np.asarray(solve(Csr.from_csr_arrays((n, n), rp, ci, v), Dense.from_columns(b), order="nd").get_col(0)).copy()
    x1 = np.asarray(solve(Csr.from_csr_arrays((n, n), rp, ci, v), Dense.from_columns(b), order="nd").get_col(0)).copy()
    assert np.array_equal(x0.view(np.uint8), x1.view(np.uint8))
    monkeypatch.delenv("BSM_ND_CACHE")
    A = Csr.from_csr_arrays((n, n), rp, ci, v)
    solve(A, Dense.from_columns(b), order="nd")
    x2 = np.asarray(solve(A, Dense.from_columns(b), order="nd").get_col(0)).copy()
    assert np.array_equal(x0.view(np.uint8), x2.view(np.uint8))
    ex = orc.solve(n, rp, ci, v, b, band=True)[0]
    assert rel_err(x0, ex) < 1e-10


def banded_spd(g, offsets):
    """n = g^2, diagonal 5, -1 on the given off-diagonals (both sides):
    strictly diagonally dominant, so SPD; sorted columns."""
    import scipy.sparse as sp

    n = g * g
    diags = [np.full(n, 5.0)] + [np.full(n - o, -1.0) for o in offsets for _ in (0, 1)]
    offs = [0] + [s * o for o in offsets for s in (1, -1)]
    m = sp.diags(diags, offs, shape=(n, n), format="csr")
    m.sort_indices()
    return m.indptr.astype(np.uint64), m.indices.astype(np.uint64), m.data.astype(np.float64)


def test_nd_plan_shared_across_handles(orc, monkeypatch):
    """solve takes `a` by value (lib.rs:11): a drop-in caller makes a new
    handle per call. A new handle with a pattern solved before reuses the
    library-wide cached plan (a hit, no analysis) and solves ITS values:
    within the tolerance of the oracle and bit-equal to a solve that builds
    its own plan (BSM_ND_SHARED=0)."""
    from basic_sparse_matrix_amd import _lib

    _lib.nd_cache_clear()
    g = 40
    n = g * g
    rp, ci, v = orc.poisson2d(g)
    b = orc.gen_x_cols(1014, n, 2)
    i0 = _lib.nd_cache_info()
    solve(Csr.from_csr_arrays((n, n), rp, ci, v), Dense.from_columns(b), order="nd")
    i1 = _lib.nd_cache_info()
    assert i1["entries"] == 1 and i1["misses"] == i0["misses"] + 1 and i1["hits"] == i0["hits"]
    v2 = 1.5 * v  # same pattern, other values
    x = solve(Csr.from_csr_arrays((n, n), rp, ci, v2), Dense.from_columns(b), order="nd")
    i2 = _lib.nd_cache_info()
    assert i2["hits"] == i1["hits"] + 1 and i2["entries"] == 1 and i2["kept_bytes"] > 0
    ex = orc.solve(n, rp, ci, v2, b, band=True)
    for j in range(2):
        assert rel_err(x.get_col(j), ex[j]) < 1e-10, j
    monkeypatch.setenv("BSM_ND_SHARED", "0")
    x_own = solve(Csr.from_csr_arrays((n, n), rp, ci, v2), Dense.from_columns(b), order="nd")
    assert _lib.nd_cache_info()["hits"] == i2["hits"]
    for j in range(2):
        assert np.array_equal(np.asarray(x.get_col(j)).view(np.uint8), np.asarray(x_own.get_col(j)).view(np.uint8))


def test_nd_plan_cache_pattern_miss_confirmed(monkeypatch):
    """Two patterns with the same n and nnz whose keys are forced to collide
    (BSM_ND_HASH_ZERO=1): the comparison of the patterns themselves rejects
    the cached plan (a miss, a new analysis), and both solve right."""
    from basic_sparse_matrix_amd import _lib

    _lib.nd_cache_clear()
    monkeypatch.setenv("BSM_ND_HASH_ZERO", "1")
    g = 24
    n = g * g
    rp1, ci1, v1 = banded_spd(g, [1, g])
    rp2, ci2, v2 = banded_spd(g, [2, g - 1])
    assert ci1.size == ci2.size and not np.array_equal(ci1, ci2)
    rng = np.random.default_rng(3)
    b = rng.uniform(-1, 1, n)
    i0 = _lib.nd_cache_info()
    for rp, ci, v in ((rp1, ci1, v1), (rp2, ci2, v2), (rp1, ci1, v1)):
        x = solve(Csr.from_csr_arrays((n, n), rp, ci, v), Dense.from_columns([b]), order="nd").get_col(0)
        a = np.zeros((n, n))
        a[np.repeat(np.arange(n), np.diff(rp.astype(np.int64))), ci.astype(np.int64)] = v
        assert rel_err(x, np.linalg.solve(a, b)) < 1e-12
    i1 = _lib.nd_cache_info()
    # pattern 1 misses, pattern 2 collides and is rejected (its plan replaces
    # pattern 1's under the shared key), pattern 1 again is rejected likewise
    assert i1["misses"] == i0["misses"] + 3 and i1["hits"] == i0["hits"]


def test_nd_plan_cache_bounded(orc, monkeypatch):
    """At most BSM_ND_CACHE_ENTRIES patterns; with BSM_ND_CACHE_MB=0 only the
    plan just used keeps its numeric storage; bsm_nd_cache_clear empties it."""
    from basic_sparse_matrix_amd import _lib

    _lib.nd_cache_clear()
    monkeypatch.setenv("BSM_ND_CACHE_ENTRIES", "2")
    monkeypatch.setenv("BSM_ND_CACHE_MB", "0")
    kept = []
    for g in (20, 21, 22):
        n = g * g
        rp, ci, v = orc.poisson2d(g)
        solve(Csr.from_csr_arrays((n, n), rp, ci, v), Dense.from_columns(orc.gen_x_cols(1015, n, 1)), order="nd")
        info = _lib.nd_cache_info()
        kept.append(info["kept_bytes"])
        assert info["entries"] == min(len(kept), 2)
    assert 0 < kept[-1] < kept[0] + kept[1] + kept[2]
    _lib.nd_cache_clear()
    assert _lib.nd_cache_info()["entries"] == 0


@pytest.mark.parametrize("switch", ["BSM_ND_PAD_SKIP", "BSM_ND_EXT_MERGE", "BSM_ND_FWD_TILES", "BSM_ND_BWD_TILES",
                                    "BSM_ND_FRONT_NT", "BSM_ND_LAG", "BSM_ND_PULL", "BSM_ND_ZSKIP",
                                    "BSM_ND_APULL", "BSM_ND_PDESC"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("leaf", ["8", "100", "192"])
def test_nd_shortcuts_same_bits(orc, monkeypatch, switch, dtype, leaf):
    """Two shortcuts that must not change a bit, each against its switch set
    to 0 (a fresh handle per run: no cached plan or buffers shared):
    * BSM_ND_PAD_SKIP: a front's last pivot tile ends in identity padding
      when np is not a multiple of 64; its factor skips the padding's
      16-column panels, which would only reproduce that identity;
    * BSM_ND_EXT_MERGE: both children's update blocks go into the parent in
      one launch (child 0's column, then child 1's, on one wave) instead of
      one launch per child: the same adds in the same order;
    * BSM_ND_FWD_TILES: the forward solve by tile rows (one wave per node,
      tile row and column, pivot tiles' y published by flags) instead of one
      workgroup per node and column: per row the same operations in the
      same order;
    * BSM_ND_BWD_TILES: the backward solve by pivot tiles (one workgroup per
      node, pivot tile and column; the front rows' products first, then each
      pivot tile's as its x arrives) instead of one workgroup per node and
      column, which sums its rows in that same tile order;
    * BSM_ND_FRONT_NT (off by default; 4 here): fronts of at most 4 tile rows
      factored whole by one workgroup, their tiles in column order, instead
      of one ticketed workgroup per tile: every tile the same operations in
      the same order;
    * BSM_ND_LAG (512 by default; 1 here, as this size's levels have fewer
      fronts): a front's tiles below the diagonal taken right after the next
      front's diagonal tile instead of after the column's last one: the same
      tiles, only their tickets' order changes;
    * BSM_ND_PULL: the children's update blocks added inside the parent's
      nd_factor tiles (staged in LDS, the lower-level child first, then
      slot 0) instead of by nd_extend2 launches after each level: the same
      adds in the same order;
    * BSM_ND_ZSKIP: the tiles no entry of A lands in start from zero in
      the factor, neither zeroed before nor read, instead of zeroed and
      read: the same values;
    * BSM_ND_APULL: every factor tile stages its own entries of A (and the
      padding pivots' 1) from the plan's per-tile lists, instead of the
      fronts being zeroed and A assembled into them: the same values;
    * BSM_ND_PDESC: the pull reads its children's blocks from per-task
      descriptors built once per plan, instead of through the node, the
      child and the bounds: the same blocks.
    (At this size every level has fewer fronts than CUs, so the default runs
    the tile kernels on every level.)"""
    monkeypatch.setenv("BSM_ND_LEAF", leaf)
    if switch == "BSM_ND_FRONT_NT":  # off by default: on (4) against off
        monkeypatch.setenv(switch, "4")
    if switch == "BSM_ND_LAG":
        monkeypatch.setenv(switch, "1")
    g = 90
    n = g * g
    rp, ci, v = orc.poisson2d(g)
    v = v.astype(dtype)
    b = orc.gen_x_cols(1013, n, 2, dtype=dtype)
    x_skip = solve(Csr.from_csr_arrays((n, n), rp, ci, v), Dense.from_columns(b), order="nd")
    monkeypatch.setenv(switch, "0")
    x_full = solve(Csr.from_csr_arrays((n, n), rp, ci, v), Dense.from_columns(b), order="nd")
    for j in range(2):
        a0, a1 = np.asarray(x_skip.get_col(j)), np.asarray(x_full.get_col(j))
        assert np.array_equal(a0.view(np.uint8), a1.view(np.uint8)), j


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
@pytest.mark.parametrize("leaf", ["8", "100", "192"])
def test_nd_poisoned_fronts_same_bits(orc, monkeypatch, dtype, leaf):
    """With the fronts filled with NaN before the solve (BSM_ND_POISON=1),
    the default path (only the tiles A's entries land in zeroed; the others
    start from zero in the factor and are never read) gives the bits of the
    path that zeroes and reads every tile: nothing reads a tile it did not
    zero or write."""
    monkeypatch.setenv("BSM_ND_LEAF", leaf)
    g = 90
    n = g * g
    rp, ci, v = orc.poisson2d(g)
    v = v.astype(dtype)
    b = orc.gen_x_cols(1021, n, 2, dtype=dtype)
    monkeypatch.setenv("BSM_ND_POISON", "1")
    a = Csr.from_csr_arrays((n, n), rp, ci, v)
    x_p = solve(a, Dense.from_columns(b), order="nd")
    x_p2 = solve(a, Dense.from_columns(b), order="nd")  # the kept fronts, poisoned again
    monkeypatch.setenv("BSM_ND_POISON", "0")
    monkeypatch.setenv("BSM_ND_ZSKIP", "0")
    x_z = solve(Csr.from_csr_arrays((n, n), rp, ci, v), Dense.from_columns(b), order="nd")
    for j in range(2):
        a0, a1, a2 = (np.asarray(x.get_col(j)) for x in (x_p, x_p2, x_z))
        assert np.all(np.isfinite(a0))
        assert np.array_equal(a0.view(np.uint8), a2.view(np.uint8)), j
        assert np.array_equal(a1.view(np.uint8), a2.view(np.uint8)), j


def _irregular_systems(orc, kind):
    """(n, rp, ci, v) of a random SPD, a block-diagonal (separator-free
    splits, pivot-free fronts) or a 3-D Laplacian system."""
    if kind == "random":
        rng = np.random.default_rng(11)
        n = 400
        a = np.zeros((n, n))
        mask = rng.random((n, n)) < 0.015
        a[mask] = rng.uniform(-1.0, 1.0, (n, n))[mask]
        a = np.tril(a, -1)
        a = a + a.T
        a[np.arange(n), np.arange(n)] = np.abs(a).sum(axis=1) + 1.0
        rp, ci, v = csr_arrays(a)
        return n, rp, ci, v
    if kind == "blocks":
        import scipy.sparse as sp

        g = 14
        rp, ci, v = orc.poisson2d(g)
        P = sp.csr_matrix((v, ci.astype(np.int64), rp.astype(np.int64)), shape=(g * g, g * g))
        M = sp.block_diag([P, 2.0 * P, sp.identity(7) * 3.0], format="csr")
        M.sort_indices()
        return M.shape[0], M.indptr.astype(np.uint64), M.indices.astype(np.uint64), M.data.astype(np.float64)
    rp, ci, v = poisson3d(11)
    return 11 ** 3, rp.astype(np.uint64), ci, v


@pytest.mark.parametrize("kind", ["random", "blocks", "poisson3d"])
@pytest.mark.parametrize("leaf", ["4", "16", "64"])
def test_nd_poisoned_fronts_irregular_trees(orc, monkeypatch, kind, leaf):
    """Irregular separator trees (a random graph, disconnected blocks with
    pivot-free fronts, a 3-D mesh) with the fronts NaN-poisoned: the pulled
    extend-add and the zero-skip give the bits of the round-5 path (the
    extend launches, every tile zeroed and read), and x solves the system."""
    n, rp, ci, v = _irregular_systems(orc, kind)
    monkeypatch.setenv("BSM_ND_LEAF", leaf)
    b = orc.gen_x_cols(1031, n, 2)
    monkeypatch.setenv("BSM_ND_POISON", "1")
    x_p = solve(Csr.from_csr_arrays((n, n), rp, ci, v), Dense.from_columns(b), order="nd")
    monkeypatch.setenv("BSM_ND_POISON", "0")
    monkeypatch.setenv("BSM_ND_PULL", "0")
    x_r = solve(Csr.from_csr_arrays((n, n), rp, ci, v), Dense.from_columns(b), order="nd")
    ex = orc.solve(n, rp, ci, v, b, band=kind == "poisson3d")
    for j in range(2):
        a0, a1 = np.asarray(x_p.get_col(j)), np.asarray(x_r.get_col(j))
        assert np.array_equal(a0.view(np.uint8), a1.view(np.uint8)), j
        assert rel_err(a0, ex[j]) < 1e-10


@pytest.mark.parametrize("kind", ["poisson2d", "random", "blocks", "poisson3d"])
@pytest.mark.parametrize("leaf", ["4", "64", "192"])
@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_nd_folded_forward(orc, monkeypatch, kind, leaf, dtype):
    """One right-hand side: the forward solve folded into the factor's
    diagonal tiles (BSM_ND_FOLD, default) against the separate forward pass
    (BSM_ND_FOLD=0), with the fronts NaN-poisoned: another summation order,
    so within rounding (f64 1e-12, f32 1e-4 relative), and against the
    oracle; two fresh runs of the folded form give the same bits."""
    if kind == "poisson2d":
        g = 60
        n = g * g
        rp, ci, v = orc.poisson2d(g)
    else:
        n, rp, ci, v = _irregular_systems(orc, kind)
    v = v.astype(dtype)
    monkeypatch.setenv("BSM_ND_LEAF", leaf)
    monkeypatch.setenv("BSM_ND_CACHE", "0")
    b = orc.gen_x_cols(1041, n, 1, dtype=dtype)
    monkeypatch.setenv("BSM_ND_POISON", "1")
    x1 = np.asarray(solve(Csr.from_csr_arrays((n, n), rp, ci, v), Dense.from_columns(b), order="nd").get_col(0))
    x2 = np.asarray(solve(Csr.from_csr_arrays((n, n), rp, ci, v), Dense.from_columns(b), order="nd").get_col(0))
    monkeypatch.setenv("BSM_ND_FOLD", "0")
    x0 = np.asarray(solve(Csr.from_csr_arrays((n, n), rp, ci, v), Dense.from_columns(b), order="nd").get_col(0))
    assert np.all(np.isfinite(x1))
    assert np.array_equal(x1.view(np.uint8), x2.view(np.uint8))
    tol = 1e-12 if dtype == np.float64 else 1e-4
    assert rel_err(x1, x0) < tol
    if dtype == np.float64:
        ex = orc.solve(n, rp, ci, v, b, band=kind in ("poisson2d", "poisson3d"))[0]
        assert rel_err(x1, ex) < 1e-10


def test_nd_one_and_several_right_hand_sides_agree(orc, monkeypatch):
    """k = 1 takes the folded forward solve, k = 3 the separate pass: every
    column of a three-column solve agrees with its one-column solve within
    rounding (and both with the oracle)."""
    monkeypatch.setenv("BSM_ND_LEAF", "64")
    g = 50
    n = g * g
    rp, ci, v = orc.poisson2d(g)
    b = orc.gen_x_cols(1051, n, 3)
    A = Csr.from_csr_arrays((n, n), rp, ci, v)
    x3 = solve(A, Dense.from_columns(b), order="nd")
    ex = orc.solve(n, rp, ci, v, b, band=True)
    for j in range(3):
        x1 = np.asarray(solve(A, Dense.from_columns([b[j]]), order="nd").get_col(0))
        xj = np.asarray(x3.get_col(j))
        assert rel_err(x1, xj) < 1e-12
        assert rel_err(x1, ex[j]) < 1e-10


def poisson3d(g):
    """7-point Laplacian on a g^3 grid (natural order, band g^2), diagonal 6.5."""
    n = g ** 3
    idx = np.arange(n).reshape(g, g, g)
    rows, cols, vals = [idx.ravel()], [idx.ravel()], [np.full(n, 6.5)]
    for ax in range(3):
        a = np.take(idx, range(g - 1), axis=ax).ravel()
        b = np.take(idx, range(1, g), axis=ax).ravel()
        rows += [a, b]
        cols += [b, a]
        vals += [np.full(a.size, -1.0), np.full(a.size, -1.0)]
    r, c, v = np.concatenate(rows), np.concatenate(cols), np.concatenate(vals)
    o = np.lexsort((c, r))
    r, c, v = r[o], c[o], v[o]
    rp = np.concatenate([[0], np.cumsum(np.bincount(r, minlength=n))]).astype(np.uint64)
    return rp, c.astype(np.uint64), v


@pytest.mark.parametrize("g", [8, 20])
def test_nd_poisson3d_vs_oracle(orc, g):
    """A 3-D mesh (separators ~ n^(2/3): larger fronts per level than 2-D)."""
    rp, ci, v = poisson3d(g)
    n = g ** 3
    b = orc.gen_x_cols(1012, n, 2)
    x = solve(Csr.from_csr_arrays((n, n), rp, ci, v), Dense.from_columns(b), order="nd")
    ex = orc.solve(n, rp, ci, v, b, band=True)
    for j in range(2):
        assert rel_err(x.get_col(j), ex[j]) < 1e-10, j


@pytest.mark.slow
def test_c5_nd_poisson_1m_f64_properties(orc, golden_c5):
    """C5 (N = 1M): within 1e-6 relative (BASELINE.json) of the band
    oracle's exact x (sampled from tests/golden/c5_poisson_1000.json) and of
    x_true, residual tiny."""
    g = 1000
    n = g * g
    rp, ci, v = orc.poisson2d(g)
    A = Csr.from_csr_arrays((n, n), rp, ci, v)
    x_true = orc.gen_x_cols(1002, n, 1)[0]
    rows = np.repeat(np.arange(n), np.diff(rp.astype(np.int64)))
    b = np.zeros(n)
    np.add.at(b, rows, v * x_true[ci.astype(np.int64)])
    x = solve(A, Dense.from_columns([b]), order="nd").get_col(0)
    exact = np.asarray([int(h, 16) for h in golden_c5["x_sample_bits"]], dtype=np.uint64).view(np.float64)
    assert rel_err(x[::golden_c5["x_stride"]], exact) < 1e-6
    assert rel_err(x, x_true) < 1e-6
    assert residual(rp, ci, v, x, b) < 1e-12


def test_nd_plan_cache_concurrent_handles(orc):
    """Four threads, each solving a new handle of one pattern three times
    (ctypes releases the GIL, so the calls overlap): the library-wide cache's
    lookups, insertions and the kept numeric storage (one solve holds it, a
    concurrent one allocates its own) give every call the single-thread
    bits."""
    import threading

    from basic_sparse_matrix_amd import _lib

    _lib.nd_cache_clear()
    g = 48
    n = g * g
    rp, ci, v = orc.poisson2d(g)
    b = orc.gen_x_cols(1016, n, 1)
    ref = np.asarray(solve(Csr.from_csr_arrays((n, n), rp, ci, v), Dense.from_columns(b), order="nd").get_col(0)).copy()
    _lib.nd_cache_clear()
    out, errs = [], []

    def work():
        try:
            for _ in range(3):
                x = solve(Csr.from_csr_arrays((n, n), rp, ci, v), Dense.from_columns(b), order="nd").get_col(0)
                out.append(np.asarray(x).copy())
        except Exception as e:  # noqa: BLE001 -- reported below
            errs.append(repr(e))

    ts = [threading.Thread(target=work) for _ in range(4)]
    for t in ts:
        t.start()
    for t in ts:
        t.join()
    assert not errs, errs
    assert len(out) == 12
    for x in out:
        assert np.array_equal(x.view(np.uint8), ref.view(np.uint8))
    assert _lib.nd_cache_info()["entries"] == 1


def test_nd_plan_shared_across_dtypes(orc):
    """A plan serves both value types of one pattern (its numeric storage is
    re-sized per dtype): f64, then f32, then f64 again on new handles, each
    right for its own type, the f64 bits repeated."""
    from basic_sparse_matrix_amd import _lib

    _lib.nd_cache_clear()
    g = 36
    n = g * g
    rp, ci, v = orc.poisson2d(g)
    b64 = orc.gen_x_cols(1017, n, 1)
    b32 = [c.astype(np.float32) for c in b64]
    x0 = np.asarray(solve(Csr.from_csr_arrays((n, n), rp, ci, v), Dense.from_columns(b64), order="nd").get_col(0)).copy()
    x32 = solve(Csr.from_csr_arrays((n, n), rp, ci, v.astype(np.float32)), Dense.from_columns(b32), order="nd").get_col(0)
    x1 = np.asarray(solve(Csr.from_csr_arrays((n, n), rp, ci, v), Dense.from_columns(b64), order="nd").get_col(0)).copy()
    info = _lib.nd_cache_info()
    assert info["entries"] == 1 and info["hits"] >= 2
    ex = orc.solve(n, rp, ci, v, b64, band=True)[0]
    assert rel_err(x0, ex) < 1e-10
    assert rel_err(x32, ex) < 2e-3
    assert np.array_equal(x0.view(np.uint8), x1.view(np.uint8))
