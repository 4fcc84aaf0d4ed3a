"""GPU parity at the BASELINE.json configurations.

C2: 1M x 1M, 10 nnz/row, k=1 (SpMV); C3: same A, k=32 (SpMM); C4: 10M x 10M,
1000 nnz/row, k=32 -- checked on a row sample plus size-independent
properties, since the full C4 oracle run is ~1 h of CPU. Inputs come from
the device generator, which is first shown to equal the host restatement
integer for integer.
"""

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from basic_sparse_matrix_amd import _lib  # noqa: E402

pytestmark = pytest.mark.gpu


def _dev():
    from basic_sparse_matrix_amd import device

    return device


def test_device_generator_matches_host(orc):
    device = _dev()
    for (rows, n_cols, kind, a, b, vk, dt) in [
        (5000, 100_000, orc.ROWLEN_CONST, 10, 10, orc.VAL_UNIFORM, np.float64),
        (3000, 5000, orc.ROWLEN_UNIFORM, 0, 1200, orc.VAL_SMALLINT, np.int32),
        (400, 1500, orc.ROWLEN_UNIFORM, 1000, 1500, orc.VAL_UNIFORM, np.float32),  # bump passes
        (1024, 1024, orc.ROWLEN_BINOMIAL, round(0.01 * 2 ** 32), 0, orc.VAL_UNIFORM, np.float64),  # C1
    ]:
        blk = device.DeviceCsrBlock.generate(1000, 777, rows, n_cols, kind, a, b, vk, dt)
        rp = orc.gen_row_ptr(1000, rows + 777, n_cols, kind, a, b)
        rp = (rp[777:] - rp[777]).astype(np.int64)
        assert np.array_equal(blk.row_ptr.cpu().numpy(), rp)
        full_rp = orc.gen_row_ptr(1000, rows + 777, n_cols, kind, a, b)
        ci, v = orc.gen_entries(1000, full_rp, n_cols, vk, r0=777, r1=777 + rows)
        lo = int(full_rp[777])
        assert np.array_equal(blk.col.cpu().numpy().astype(np.uint64), ci[lo:])
        assert np.array_equal(blk.vals.cpu().numpy(), v[lo:].astype(dt))
        cols = ci[lo:].astype(np.int64)
        # strictly increasing inside every row, within [0, n_cols)
        inside = np.ones(max(0, len(cols) - 1), dtype=bool)
        b = rp[1:-1]
        inside[b[(b > 0) & (b < len(cols))] - 1] = False
        assert (np.diff(cols)[inside] > 0).all() and cols.min() >= 0 and cols.max() < n_cols
    x = device.gen_dense(1001, 5, 1000, 7)
    ex = np.stack(orc.gen_x_cols(1001, 1005, 7), axis=1)[5:]
    assert np.array_equal(x.cpu().numpy(), ex)


def _run_spmm(blk, x, k):
    device = _dev()
    y = torch.empty((blk.rows, k), dtype=torch.float64, device="cuda")
    row_nnz = torch.empty(blk.rows, dtype=torch.int32, device="cuda")
    blk.spmm(x, y, row_nnz)
    comp = device.Compactor(blk.rows, k, np.float64)
    comp(y, row_nnz)
    torch.cuda.synchronize()
    return y, comp


def test_c1_public_api_bit_exact(orc):
    """C1 (BASELINE.json configs[0]): 1024 x 1024, Binomial(1024, 0.01) row
    lengths (~10.5k nnz, some rows empty or long), k = 1, f64, through the
    public Csr.mul_dense (sparse.rs:426-446) with host operands, bit-exact
    against the oracle; then the same matrix through the device-level SpMV
    (the bench's timed path) and compaction."""
    from basic_sparse_matrix_amd import Csr, Dense

    rows = n_cols = 1024
    rp = orc.gen_row_ptr(1000, rows, n_cols, orc.ROWLEN_BINOMIAL, round(0.01 * 2 ** 32), 0)
    ci, v = orc.gen_entries(1000, rp, n_cols)
    lens = np.diff(rp.astype(np.int64))
    assert 9_000 < rp[-1] < 12_000 and lens.min() <= 3 and lens.max() >= 18
    x_cols = orc.gen_x_cols(1001, n_cols, 1)
    got = Csr.from_csr_arrays((rows, n_cols), rp, ci, v).mul_dense(Dense.from_columns(x_cols))
    erp, eci, ev = orc.mul_dense(rows, n_cols, rp, ci, v, x_cols)
    assert np.array_equal(np.asarray(got.row_index, np.uint64), erp)
    assert np.array_equal(np.asarray(got.col_index, np.uint64), eci)
    assert np.array_equal(np.asarray(got.v).view(np.uint64), ev.view(np.uint64))
    device = _dev()
    blk = device.DeviceCsrBlock.generate(1000, 0, rows, n_cols, _lib.ROWLEN_BINOMIAL, round(0.01 * 2 ** 32), 0)
    y, comp = _run_spmm(blk, device.gen_dense(1001, 0, n_cols, 1), 1)
    assert np.array_equal(comp.row_ptr.cpu().numpy(), erp.astype(np.int64))
    assert np.array_equal(comp.vals[:comp.nnz()].cpu().numpy().view(np.uint64), ev.view(np.uint64))


# default / spmv_stream / spmv_wave / spmv_thread (the default for few short rows)
@pytest.mark.parametrize("variant", ["0", "1", "5", "6"])
def test_spmv_variants_ragged_rows_bit_exact(orc, monkeypatch, variant):
    """k = 1 on ragged rows (empty rows, rows longer than a workgroup's LDS
    chunk) through every SpMV kernel, bit-exact."""
    from basic_sparse_matrix_amd import Csr, Dense

    monkeypatch.setenv("BSM_SPMV_VARIANT", variant)
    rows, n_cols = 3000, 50_000
    lens = np.random.default_rng(7).integers(0, 12, rows)
    lens[[5, 700, 2999]] = [0, 9000, 5000]  # rows longer than 256 * 16 entries
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    ci, v = orc.gen_entries(1000, rp, n_cols)
    x_cols = orc.gen_x_cols(1001, n_cols, 1)
    got = Csr.from_csr_arrays((rows, n_cols), rp, ci, v).mul_dense(Dense.from_columns(x_cols))
    erp, eci, ev = orc.mul_dense(rows, n_cols, rp, ci, v, x_cols)
    assert np.array_equal(np.asarray(got.row_index, np.uint64), erp)
    assert np.array_equal(np.asarray(got.v).view(np.uint64), ev.view(np.uint64))


@pytest.mark.parametrize("k", [1, 32])
def test_c2_c3_full_size_bit_exact(orc, k):
    """C2 (k=1) and C3 (k=32) at full size, every output element checked."""
    device = _dev()
    rows = n_cols = 1_000_000
    blk = device.DeviceCsrBlock.generate(1000, 0, rows, n_cols, _lib.ROWLEN_CONST, 10, 10)
    x = device.gen_dense(1001, 0, n_cols, k)
    y, comp = _run_spmm(blk, x, k)
    rp = orc.gen_row_ptr(1000, rows, n_cols, orc.ROWLEN_CONST, 10, 10)
    ci, v = orc.gen_entries(1000, rp, n_cols)
    x_cols = orc.gen_x_cols(1001, n_cols, k)
    erp, eci, ev = orc.mul_dense(rows, n_cols, rp, ci, v, x_cols)
    assert np.array_equal(comp.row_ptr.cpu().numpy(), erp.astype(np.int64))
    n = comp.nnz()
    assert np.array_equal(comp.col[:n].cpu().numpy().astype(np.uint64), eci)
    assert np.array_equal(comp.vals[:n].cpu().numpy().view(np.uint64), ev.view(np.uint64))


def test_c4_shape_sampled_rows(orc):
    """C4 shape (10M columns, 1000 nnz/row, k=32) on a 4k-row block taken
    from the middle of the 10M rows: every output of the block is compared
    bit-exactly with the oracle."""
    device = _dev()
    n_cols, k, row0, rows = 10_000_000, 32, 4_321_000, 4_000
    blk = device.DeviceCsrBlock.generate(1000, row0, rows, n_cols, _lib.ROWLEN_CONST, 1000, 1000)
    x = device.gen_dense(1001, 0, n_cols, k)
    y, comp = _run_spmm(blk, x, k)
    rp = np.arange(rows + 1, dtype=np.uint64) * 1000
    full = np.zeros(row0 + rows + 1, dtype=np.uint64)
    full[row0:] = rp  # only rows [row0, row0+rows) are generated
    ci, v = orc.gen_entries(1000, full, n_cols, r0=row0, r1=row0 + rows)
    x_cols = orc.gen_x_cols(1001, n_cols, k)
    erp, eci, ev = orc.mul_dense(rows, n_cols, rp, ci, v, x_cols)
    assert np.array_equal(comp.row_ptr.cpu().numpy(), erp.astype(np.int64))
    n = comp.nnz()
    assert n == rows * k  # positive inputs: nothing is dropped
    assert np.array_equal(comp.vals[:n].cpu().numpy().view(np.uint64), ev.view(np.uint64))
    # the column-panel schedule bench.py uses at C4 (default width) gives the same bits
    assert blk.plan(k) == 2_000_000
    y2, comp2 = _run_spmm(blk, x, k)
    assert torch.equal(y2.view(torch.int64), y.view(torch.int64))
    assert torch.equal(comp2.row_ptr, comp.row_ptr)


def test_c4_full_size_two_schedules_and_oracle_samples(orc):
    """C4 at full size (10M x 10M, 1e10 nnz, k = 32, f64): the tiled copy the
    bench times and the one-pass row kernel (a different schedule, each
    bit-exact against the oracle on blocks) give the same bits for all 320M
    outputs, and 256 rows spread over the 10M match the oracle bit for bit.
    Needs ~250 GB of HBM (A 120 GB + the tiled copy 124 GB + X + Y)."""
    import gc

    device = _dev()
    rows = n_cols = 10_000_000
    k, nnz_r = 32, 1000
    if torch.cuda.mem_get_info()[0] < 258 * 2**30:
        pytest.skip("needs ~258 GiB of free HBM")
    blk = device.DeviceCsrBlock.generate(1000, 0, rows, n_cols, _lib.ROWLEN_CONST, nnz_r, nnz_r)
    x = device.gen_dense(1001, 0, n_cols, k)
    assert blk.plan_tiled(k) is not None
    y_t = torch.empty((rows, k), dtype=torch.float64, device="cuda")
    blk.spmm(x, y_t)
    torch.cuda.synchronize()
    blk.tiled = None  # frees the copy
    gc.collect()
    y_p = torch.empty((rows, k), dtype=torch.float64, device="cuda")
    blk.spmm(x, y_p)  # one-pass kernel: no plan
    torch.cuda.synchronize()
    assert torch.equal(y_t.view(torch.int64), y_p.view(torch.int64))
    del y_p, blk
    gc.collect()
    rng = np.random.default_rng(4)
    sample = np.sort(np.concatenate([[0, rows - 1], rng.choice(rows, 254, replace=False)]))
    ci_l, v_l = [], []
    for r in sample:  # row r alone: zero-length rows before it
        full = np.zeros(r + 2, dtype=np.uint64)
        full[r + 1] = nnz_r
        ci, v = orc.gen_entries(1000, full, n_cols, r0=int(r), r1=int(r) + 1)
        ci_l.append(ci[:nnz_r])
        v_l.append(v[:nnz_r])
    rp = np.arange(len(sample) + 1, dtype=np.uint64) * nnz_r
    x_cols = orc.gen_x_cols(1001, n_cols, k)
    erp, eci, ev = orc.mul_dense(len(sample), n_cols, rp, np.concatenate(ci_l), np.concatenate(v_l), x_cols)
    assert np.array_equal(erp, np.arange(len(sample) + 1, dtype=np.uint64) * k)  # nothing dropped
    got = y_t[torch.as_tensor(sample, device="cuda")].cpu().numpy().reshape(-1)
    assert np.array_equal(got.view(np.uint64), ev.view(np.uint64))
