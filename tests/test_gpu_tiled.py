"""Row-block x column-panel SpMM schedule (kernels_tiled.hip): the re-laid
copy of the matrix must give the same Y and row_nnz as the one-row-per-wave
kernels, bit for bit, and the oracle's values (Csr::mul_dense,
src/sparse.rs:426-446). Cases: the C4 shape on a 2M-row block (every row
compared with the panelled kernel, a row sample with the oracle), uneven and
empty rows, rows shorter than the wave count, several batches per wave,
unsorted rows (storage-order sums), signed values with exact cancellations,
NaN/inf."""


import numpy as np
import pytest

torch = pytest.importorskip("torch")

from basic_sparse_matrix_amd import _lib  # noqa: E402

pytestmark = pytest.mark.gpu


def _dev():
    from basic_sparse_matrix_amd import device

    return device


def _spmm(blk, x, tiled):
    y = torch.full((blk.rows, x.shape[1]), float("nan"), dtype=torch.float64, device="cuda")
    nnz = torch.full((blk.rows,), -1, dtype=torch.int32, device="cuda")
    saved = blk.tiled
    if not tiled:
        blk.tiled = None
    blk.spmm(x, y, nnz)
    blk.tiled = saved
    torch.cuda.synchronize()
    return y, nnz


def _same(a, b):
    return torch.equal(a.view(torch.int64), b.view(torch.int64))


def _block(rp, ci, v, n_cols):
    device = _dev()
    return device.DeviceCsrBlock(0, len(rp) - 1, n_cols, torch.as_tensor(rp, dtype=torch.int64, device="cuda"),
                                 torch.as_tensor(ci, dtype=torch.int32, device="cuda"),
                                 torch.as_tensor(v, dtype=torch.float64, device="cuda"), np.dtype(np.float64))


@pytest.fixture
def geometry(monkeypatch):
    def set_geometry(rw=None, waves=None, pshift=None):
        for name, val in (("BSM_TILED_RW", rw), ("BSM_TILED_WAVES", waves), ("BSM_TILED_PSHIFT", pshift)):
            if val is None:
                monkeypatch.delenv(name, raising=False)
            else:
                monkeypatch.setenv(name, str(val))

    return set_geometry


@pytest.mark.parametrize("rw,waves,pshift", [(None, None, None), (16, 64, 10), (144, 8, 6), (96, 4, 13)])
def test_tiled_equals_rowwave_random(orc, geometry, rw, waves, pshift):
    device = _dev()
    geometry(rw, waves, pshift)
    rows, n_cols, k = 30_000, 200_000, 32
    blk = device.DeviceCsrBlock.generate(1000, 0, rows, n_cols, _lib.ROWLEN_UNIFORM, 0, 120)  # empty rows too
    x = device.gen_dense(1001, 0, n_cols, k)
    assert blk.plan_tiled(k, force=True) is not None
    y1, n1 = _spmm(blk, x, tiled=True)
    y0, n0 = _spmm(blk, x, tiled=False)
    assert _same(y1, y0) and torch.equal(n1, n0)
    info = blk.tiled.info()
    assert info["slots"] >= blk.nnz and info["panel_cols"] == 1 << (pshift or 12)
    # a row sample against the oracle
    rp = blk.row_ptr.cpu().numpy().astype(np.uint64)
    ci, v = blk.col.cpu().numpy(), blk.vals.cpu().numpy()
    r0, r1 = 12_345, 12_645
    sub_rp = (rp[r0:r1 + 1] - rp[r0]).astype(np.uint64)
    x_cols = orc.gen_x_cols(1001, n_cols, k)
    erp, eci, ev = orc.mul_dense(r1 - r0, n_cols, sub_rp, ci[rp[r0]:rp[r1]], v[rp[r0]:rp[r1]], x_cols)
    got = y1[r0:r1].cpu().numpy()
    dense = np.zeros((r1 - r0, k))
    for r in range(r1 - r0):
        dense[r, eci[erp[r]:erp[r + 1]]] = ev[erp[r]:erp[r + 1]]
    assert np.array_equal(got.view(np.uint64), dense.view(np.uint64))


def test_tiled_tiny_and_uneven(geometry):
    """Fewer rows than waves, one long row among short ones, empty matrix rows."""
    geometry(None, 64, 8)
    rng = np.random.default_rng(7)
    n_cols, k = 5000, 32
    lens = rng.integers(0, 6, size=50)
    lens[17] = 3000  # long row: serialised one entry per chunk
    lens[3] = 0
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    ci = np.concatenate([np.sort(rng.choice(n_cols, size=n, replace=False)) for n in lens]).astype(np.int32)
    v = rng.standard_normal(rp[-1])
    blk = _block(rp, ci, v, n_cols)
    x = torch.as_tensor(rng.standard_normal((n_cols, k)), device="cuda")
    assert blk.plan_tiled(k, force=True) is not None
    y1, n1 = _spmm(blk, x, True)
    y0, n0 = _spmm(blk, x, False)
    assert _same(y1, y0) and torch.equal(n1, n0)


def test_tiled_unsorted_rows_keep_storage_order(geometry):
    """Columns in random order inside each row: the layout takes every row's
    entries in storage order, so the sums match the in-order kernel."""
    geometry(32, 16, 9)
    rng = np.random.default_rng(11)
    rows, n_cols, k = 3000, 40_000, 32
    lens = rng.integers(1, 80, size=rows)
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    ci = np.concatenate([rng.permutation(rng.choice(n_cols, size=n, replace=False)) for n in lens]).astype(np.int32)
    v = rng.standard_normal(rp[-1]) * 1e3
    blk = _block(rp, ci, v, n_cols)
    x = torch.as_tensor(rng.standard_normal((n_cols, k)), device="cuda")
    assert blk.plan_tiled(k, force=True) is not None
    y1, n1 = _spmm(blk, x, True)
    y0, n0 = _spmm(blk, x, False)
    assert _same(y1, y0) and torch.equal(n1, n0)


def test_tiled_cancellation_zero_pattern_nan_inf(geometry):
    """Small integers with exact cancellations (zeros that compaction drops),
    -0.0 inputs, NaN and inf in X: the same bits and counts."""
    geometry(24, 8, 7)
    rng = np.random.default_rng(5)
    rows, n_cols, k = 2000, 3000, 32
    lens = rng.integers(0, 40, size=rows)
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    ci = np.concatenate([np.sort(rng.choice(n_cols, size=n, replace=False)) for n in lens]).astype(np.int32)
    v = rng.integers(-3, 4, size=rp[-1]).astype(np.float64)
    v[v == 0] = -0.0
    xs = rng.integers(-2, 3, size=(n_cols, k)).astype(np.float64)
    xs[7, 3] = np.nan
    xs[11, :] = np.inf
    blk = _block(rp, ci, v, n_cols)
    x = torch.as_tensor(xs, device="cuda")
    assert blk.plan_tiled(k, force=True) is not None
    y1, n1 = _spmm(blk, x, True)
    y0, n0 = _spmm(blk, x, False)
    assert _same(y1, y0) and torch.equal(n1, n0)
    assert int((n0 < k).sum()) > 0  # the zero pattern is exercised


def test_tiled_c4_shape_block_matches_panelled(orc):
    """C4 shape (10M columns, 1000 nnz/row, k=32) on a 2M-row block with the
    library's default geometry: every row equals the column-panel kernel
    bench.py used before, and a row sample equals the oracle."""
    device = _dev()
    n_cols, k, row0, rows = 10_000_000, 32, 3_000_000, 2_000_000
    blk = device.DeviceCsrBlock.generate(1000, row0, rows, n_cols, _lib.ROWLEN_CONST, 1000, 1000)
    x = device.gen_dense(1001, 0, n_cols, k)
    assert blk.plan_tiled(k) is not None  # wanted at this shape
    y1, n1 = _spmm(blk, x, True)
    blk.tiled = None
    torch.cuda.empty_cache()
    assert blk.plan(k) == 2_000_000
    y0, n0 = _spmm(blk, x, False)
    assert _same(y1, y0) and torch.equal(n1, n0)
    assert int(n1.min()) == k
    sr = 1_234_567
    rp = np.zeros(row0 + sr + 3, dtype=np.uint64)
    rp[row0 + sr:] = np.arange(3, dtype=np.uint64) * 1000
    ci, v = orc.gen_entries(1000, rp, n_cols, r0=row0 + sr, r1=row0 + sr + 2)
    erp, eci, ev = orc.mul_dense(2, n_cols, rp[row0 + sr:] - rp[row0 + sr], ci, v, orc.gen_x_cols(1001, n_cols, k))
    assert np.array_equal(y1[sr:sr + 2].reshape(-1).cpu().numpy().view(np.uint64), ev.view(np.uint64))


def test_public_mul_dense_uses_tiled_copy(orc, monkeypatch):
    """Csr.mul_dense (the reference API) builds the tiled copy once per matrix
    when the library wants it (forced here for a small shape) and returns the
    oracle's Csr bit for bit; with the copy disabled, the same Csr."""
    import ctypes

    from basic_sparse_matrix_amd import Csr, Dense

    rows, n_cols, k = 20_000, 60_000, 32
    rp, ci, v = orc.gen_csr(1000, rows, n_cols, orc.ROWLEN_UNIFORM, 150, 250)
    x_cols = orc.gen_x_cols(1001, n_cols, k)
    monkeypatch.setenv("BSM_SPMM_TILED", "2")
    monkeypatch.setenv("BSM_TILED_WAVES", "64")
    a = Csr.from_csr_arrays((rows, n_cols), rp, ci, v)
    got = a.mul_dense(Dense.from_columns(x_cols))
    used = ctypes.c_int(-1)
    _lib.check(_lib.load().bsm_csr_tiled(a._device().handle, ctypes.byref(used)))
    assert used.value == 1
    got2 = a.mul_dense(Dense.from_columns(x_cols))  # cached copy
    erp, eci, ev = orc.mul_dense(rows, n_cols, rp, ci, v, x_cols)
    for g in (got, got2):
        assert np.array_equal(np.asarray(g.row_index), erp)
        assert np.array_equal(np.asarray(g.col_index), eci)
        assert np.array_equal(np.asarray(g.v).view(np.uint64), ev.view(np.uint64))
    monkeypatch.setenv("BSM_SPMM_TILED", "0")
    b = Csr.from_csr_arrays((rows, n_cols), rp, ci, v)
    ref = b.mul_dense(Dense.from_columns(x_cols))
    _lib.check(_lib.load().bsm_csr_tiled(b._device().handle, ctypes.byref(used)))
    assert used.value == 0
    assert np.array_equal(np.asarray(ref.v).view(np.uint64), ev.view(np.uint64))


@pytest.mark.parametrize("rw,waves,pshift", [(None, None, None), (300, 16, 12), (2047, 4, 15)])
def test_tiled_k1_equals_spmv(geometry, rw, waves, pshift):
    """k = 1 (SpMV): the copy with one LDS double per row gives the k = 1
    kernels' y and counts bit for bit (uneven and empty rows, signed values)."""
    geometry(rw, waves, pshift)
    rng = np.random.default_rng(3)
    rows, n_cols = 20_000, 300_000
    lens = rng.integers(0, 25, size=rows)
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.int64)
    ci = np.concatenate([np.sort(rng.choice(n_cols, size=n, replace=False)) for n in lens]).astype(np.int32)
    v = rng.standard_normal(rp[-1])
    blk = _block(rp, ci, v, n_cols)
    x = torch.as_tensor(rng.standard_normal((n_cols, 1)), device="cuda")
    assert blk.plan_tiled(1, force=True) is not None
    y1, n1 = _spmm(blk, x, True)
    y0, n0 = _spmm(blk, x, False)
    assert _same(y1, y0) and torch.equal(n1, n0)


def test_tiled_k1_c2_shape(orc):
    """C2 (1M x 1M, 10 nnz/row, k = 1): the library wants the copy at this
    shape; every row equals the k = 1 kernel and a sample equals the oracle."""
    device = _dev()
    rows = n_cols = 1_000_000
    blk = device.DeviceCsrBlock.generate(1000, 0, rows, n_cols, _lib.ROWLEN_CONST, 10, 10)
    x = device.gen_dense(1001, 0, n_cols, 1)
    assert blk.plan_tiled(1) is not None
    y1, n1 = _spmm(blk, x, True)
    y0, n0 = _spmm(blk, x, False)
    assert _same(y1, y0) and torch.equal(n1, n0)
    rp = blk.row_ptr.cpu().numpy().astype(np.uint64)
    ci, v = blk.col.cpu().numpy(), blk.vals.cpu().numpy()
    r0, r1 = 777_000, 778_000
    sub = (rp[r0:r1 + 1] - rp[r0]).astype(np.uint64)
    erp, eci, ev = orc.mul_dense(r1 - r0, n_cols, sub, ci[rp[r0]:rp[r1]], v[rp[r0]:rp[r1]], orc.gen_x_cols(1001, n_cols, 1))
    assert np.array_equal(y1[r0:r1, 0].cpu().numpy().view(np.uint64), ev.view(np.uint64))


@pytest.mark.parametrize("k,rw", [(32, None), (32, "100"), (1, None)])
def test_public_mul_dense_tiled_copy_f32(orc, monkeypatch, k, rw):
    """Csr<f32>.mul_dense on the tiled copy (f32 value stream, 128-B Y rows in
    LDS, up to 255 rows per batch at k = 32): the oracle's f32 Csr bit for bit
    (f32 multiply, then f32 add, in storage order), and the same Csr as the
    one-row-per-wave kernels with the copy off. Some unsorted rows, signed
    values with exact cancellations, NaN and inf included."""
    import ctypes

    from basic_sparse_matrix_amd import Csr, Dense

    rng = np.random.default_rng(21 + k)
    rows, n_cols = 12_000, 50_000
    lens = rng.integers(150, 250, size=rows)  # even enough for the copy's padding bound
    lens[::1000] = 0
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    # sorted rows, every 50th with its neighbouring entries swapped pairwise:
    # unsorted (storage-order sums) but in panel order nearly everywhere. The
    # public path takes the copy only within its padding bound, which fully
    # shuffled rows exceed (a row stalls on an early high-panel entry); those
    # are covered through the forced copy, test_tiled_unsorted_rows_keep_storage_order
    def row_cols(i, n):
        c = np.sort(rng.choice(n_cols, size=n, replace=False))
        if i % 50 == 7 and n > 1:
            m = n - n % 2
            c[:m] = c[:m].reshape(-1, 2)[:, ::-1].reshape(-1)
        return c

    ci = np.concatenate([row_cols(i, n) for i, n in enumerate(lens)]).astype(np.uint64)
    v = rng.standard_normal(int(rp[-1])).astype(np.float32)
    v[::97] = rng.integers(-3, 4, size=v[::97].size).astype(np.float32)
    x_cols = [rng.integers(-2, 3, size=n_cols).astype(np.float32) if j % 3 == 0
              else rng.standard_normal(n_cols).astype(np.float32) for j in range(k)]
    x_cols[0][5] = np.nan
    x_cols[-1][9] = np.inf
    monkeypatch.setenv("BSM_SPMM_TILED", "2")
    monkeypatch.setenv("BSM_TILED_WAVES", "64")
    if rw:
        monkeypatch.setenv("BSM_TILED_RW", rw)
    a = Csr.from_csr_arrays((rows, n_cols), rp, ci, v)
    got = a.mul_dense(Dense.from_columns(x_cols))
    used = ctypes.c_int(-1)
    _lib.check(_lib.load().bsm_csr_tiled(a._device().handle, ctypes.byref(used)))
    assert used.value == 1
    erp, eci, ev = orc.mul_dense(rows, n_cols, rp, ci, v, x_cols)
    assert np.array_equal(np.asarray(got.row_index), erp)
    assert np.array_equal(np.asarray(got.col_index), eci)
    assert np.array_equal(np.asarray(got.v).view(np.uint32), ev.view(np.uint32))
    monkeypatch.setenv("BSM_SPMM_TILED", "0")
    b = Csr.from_csr_arrays((rows, n_cols), rp, ci, v)
    ref = b.mul_dense(Dense.from_columns(x_cols))
    _lib.check(_lib.load().bsm_csr_tiled(b._device().handle, ctypes.byref(used)))
    assert used.value == 0
    assert np.array_equal(np.asarray(ref.v).view(np.uint32), ev.view(np.uint32))


def test_tiled_wanted_f32_c4_shape():
    """The library takes the tiled copy for an f32 C4-shaped product (X beyond
    1 GiB at k = 32), as for f64, and for matrices wider than 2^24 columns."""
    lib = _lib.load()
    f32, f64 = _lib.DTYPE_CODES[np.dtype(np.float32)], _lib.DTYPE_CODES[np.dtype(np.float64)]
    assert lib.bsm_dev_tiled_wanted(f32, 10_000_000, 10_000_000, 10_000_000_000, 32, 1000) == 1
    assert lib.bsm_dev_tiled_wanted(f64, 10_000_000, 10_000_000, 10_000_000_000, 32, 1000) == 1
    # 2^24 columns and more: the 64-bit meta copy; device columns are int32
    assert lib.bsm_dev_tiled_wanted(f32, 10_000_000, 1 << 24, 10_000_000_000, 32, 1000) == 1
    assert lib.bsm_dev_tiled_wanted(f64, 10_000_000, 1 << 31, 10_000_000_000, 32, 1000) == 0


def test_tiled_wide_columns_64bit_meta(geometry):
    """2^25 columns (X = 8.6 GB): the copy's meta word is 64-bit (col << 8 |
    row no longer fits 32 bits past 2^24 columns). The same Y and counts as the
    one-row-per-wave kernel, bit for bit, and a row sample summed in storage
    order on the host from the same X rows (multiply, then add, in f64)."""
    device = _dev()
    geometry(None, 256, None)
    rows, n_cols, k = 20_000, 1 << 25, 32
    blk = device.DeviceCsrBlock.generate(1000, 0, rows, n_cols, _lib.ROWLEN_UNIFORM, 40, 160)
    x = device.gen_dense(1001, 0, n_cols, k)
    assert blk.plan_tiled(k, force=True) is not None
    info = blk.tiled.info()
    assert info["bytes"] >= info["slots"] * 16  # 8-B meta + 8-B value per slot
    y1, n1 = _spmm(blk, x, True)
    y0, n0 = _spmm(blk, x, False)
    assert _same(y1, y0) and torch.equal(n1, n0)
    rp = blk.row_ptr.cpu().numpy()
    ci = blk.col.cpu().numpy()
    v = blk.vals.cpu().numpy()
    assert int(ci.max()) >= 1 << 24
    for r in (0, 777, 12_345, rows - 1):
        cols = ci[rp[r]:rp[r + 1]].astype(np.int64)
        xr = x[torch.as_tensor(cols, device="cuda")].cpu().numpy()
        acc = np.zeros(k)
        for e in range(len(cols)):
            acc = acc + v[rp[r] + e] * xr[e]  # f64 multiply, then add: the reference's order
        assert np.array_equal(y1[r].cpu().numpy().view(np.uint64), acc.view(np.uint64)), r
    del x
    torch.cuda.empty_cache()
