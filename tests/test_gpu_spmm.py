"""GPU parity of the SpMM / SpMV / transpose hot path (Csr::mul_dense,
mul_dense_s, mul_vector, transpose; src/sparse.rs:296-318, 426-482).

Every test runs the HIP path through the C-ABI (libbsm_hip.so) and compares
it with the CPU oracle (oracle/, pinned by tests/test_oracle_golden.py) or
with the reference's own golden vectors. The bar is BIT-EXACT for row_ptr,
col_idx and values, floats included: the kernels keep the reference's
per-element summation order and never contract to FMA.
"""

import numpy as np
import pytest

import basic_sparse_matrix_amd as bsm
from basic_sparse_matrix_amd import Csr, Dense, DenseS, MatErr, MatErrKind, Panic
from golden.golden_io import matrix

pytestmark = pytest.mark.gpu


def assert_csr_bits(got: Csr, rp, ci, v):
    assert got.is_finalised and got.iter_v_index == 0 and got.iter_row_index == 0
    assert np.array_equal(np.asarray(got.row_index, np.uint64), np.asarray(rp, np.uint64)), "row_ptr differs"
    assert np.array_equal(np.asarray(got.col_index, np.uint64), np.asarray(ci, np.uint64)), "col_idx differs"
    gv, ev = np.asarray(got.v), np.asarray(v, dtype=got.dtype)
    assert gv.dtype == ev.dtype and gv.shape == ev.shape
    if gv.dtype.kind == "f":
        ib = np.uint64 if gv.dtype.itemsize == 8 else np.uint32
        bad = np.nonzero(gv.view(ib) != ev.view(ib))[0]
        assert bad.size == 0, f"{bad.size} values differ, first at {bad[:5]}: {gv[bad[:5]]} vs {ev[bad[:5]]}"
    else:
        assert np.array_equal(gv, ev)


# ------------------------------------------------ reference unit tests (GPU)
def test_dense_mul_golden(golden):
    g = golden["test_dense_mul"]
    d = Dense.from_data(g["x_cols"])
    s = Csr.from_data(g["rows"])
    assert s.mul_dense(d) == Csr.from_data(g["out_rows"])  # sparse.rs:1106-1108


def test_nnz_golden(golden):
    g = golden["test_nnz"]
    out = Csr.from_data(g["rows"]).mul_dense(Dense.from_data(g["x_cols"]))
    assert out == Csr.from_data(g["out_rows"])
    assert out.get_nnz() == g["out_nnz"]  # sparse.rs:1176


@pytest.mark.parametrize("name", ["transpose_1x1", "transpose_nxn", "transpose_mxn"])
def test_transpose_golden(golden, name):
    g = golden[name]
    assert Csr.from_data(g["rows"]).transpose() == Csr.from_data(g["t_rows"])


def test_mul_vector_golden(golden):
    g = golden["test_mul_vector"]
    v = np.asarray(g["v"], dtype=np.int32)
    out = np.zeros(g["err_out_len"], dtype=np.int32)
    with pytest.raises(MatErr) as e:
        Csr.from_data(g["err_rows"]).mul_vector(v, out)
    assert e.value.kind == MatErrKind.IncorrectDimensions  # sparse.rs:1510
    Csr.from_data(g["eye_rows"]).mul_vector(v, out)
    assert list(out) == list(v)
    out2 = np.zeros(2, dtype=np.int32)
    Csr.from_data(g["rows"]).mul_vector(v, out2)
    assert list(out2) == g["out"]


def test_cholesky_transpose_golden_u(golden):
    # the transpose half of cholesky_decomposition_0 (sparse.rs:1053-1059)
    g = golden["cholesky_decomposition_0"]
    l = Csr.from_data(matrix(g["l_rows"], np.float32), dtype=np.float32)
    assert l.transpose() == Csr.from_data(matrix(g["u_rows"], np.float32), dtype=np.float32)


def test_mul_dense_dimension_error():
    a = Csr.from_data([[1, 2], [3, 4]])
    with pytest.raises(MatErr) as e:
        a.mul_dense(Dense.from_data([[1, 2, 3]]))
    assert e.value.kind == MatErrKind.IncorrectDimensions


def test_mul_dense_s_matches_mul_dense(golden):
    g = golden["test_dense_mul"]
    s = Csr.from_data(g["rows"])
    ds = DenseS.from_data(g["x_cols"])
    assert s.mul_dense_s(ds) == s.mul_dense(Dense.from_data(g["x_cols"]))
    assert s.mul_dense_s(ds) == Csr.from_data(g["out_rows"])  # the golden itself (sparse.rs:1106-1108)
    with pytest.raises(MatErr):
        s.mul_dense_s(DenseS.new_default(3, 2, np.int32))


@pytest.mark.parametrize("dtype,k", [(np.float64, 1), (np.float64, 32), (np.float32, 5), (np.int64, 3)])
def test_mul_dense_s_random_vs_oracle(orc, dtype, k):
    """mul_dense_s (sparse.rs:448-466) against the oracle's mul_dense on the
    same columns, not against the GPU's own mul_dense."""
    dt = np.dtype(dtype)
    vk = orc.VAL_UNIFORM if dt.kind == "f" else orc.VAL_SMALLINT
    rows, n_cols = 900, 400
    rp, ci, v = orc.gen_csr(300 + k, rows, n_cols, kind=orc.ROWLEN_UNIFORM, a=0, b=30, value_kind=vk, dtype=dt)
    a = Csr.from_csr_arrays((rows, n_cols), rp, ci, v)
    x_cols = orc.gen_x_cols(301 + k, n_cols, k, value_kind=vk, dtype=dt)
    ds = DenseS.from_data([list(c) for c in x_cols], dtype=dt)
    assert_csr_bits(a.mul_dense_s(ds), *orc.mul_dense(rows, n_cols, rp, ci, v, x_cols))


# ----------------------------------------------------- randomized parity
def oracle_mul_dense(orc, a: Csr, x_cols):
    rp, ci, v = a._csr_arrays()
    return orc.mul_dense(a.dims.rows, a.dims.cols, rp, ci, v, x_cols)


DTYPES = [np.float64, np.float32, np.int32, np.uint32, np.int64, np.uint64]


@pytest.mark.parametrize("dtype", DTYPES)
@pytest.mark.parametrize("k", [1, 2, 3, 10, 32, 33, 64, 65, 100])
def test_mul_dense_random_parity(orc, dtype, k):
    dt = np.dtype(dtype)
    vk = orc.VAL_UNIFORM if dt.kind == "f" else orc.VAL_SMALLINT
    rows, n_cols = 1500, 700
    rp, ci, v = orc.gen_csr(7 + k, rows, n_cols, kind=orc.ROWLEN_UNIFORM, a=0, b=40, value_kind=vk, dtype=dt)
    a = Csr.from_csr_arrays((rows, n_cols), rp, ci, v)
    x_cols = orc.gen_x_cols(11 + k, n_cols, k, value_kind=vk, dtype=dt)
    got = a.mul_dense(Dense.from_columns(x_cols))
    assert_csr_bits(got, *oracle_mul_dense(orc, a, x_cols))


@pytest.mark.parametrize("dtype", [np.float64, np.int32])
@pytest.mark.parametrize("rows,k", [(1, 1), (1024, 1), (1500, 3), (8192, 16), (8193, 1), (4096, 32), (2048, 64),
                                    (1000, 131)])
def test_small_result_host_copy_and_device_arrays(orc, monkeypatch, dtype, rows, k):
    """Small results (rows <= 8192, rows x k <= 131,072; C1's shape) are
    scanned and compacted by one workgroup that writes the result's device
    arrays AND the host copy bsm_csr_download then serves. Both must equal
    the oracle: the host copy through the download, the device arrays through
    a device transpose of the result handle (transpose results have no host
    copy). The shapes straddle both limits; BSM_SMALL_OUT=0 (scan +
    compaction launches, download copies) gives the same bits."""
    import ctypes

    from basic_sparse_matrix_amd import _lib

    dt = np.dtype(dtype)
    vk = orc.VAL_SMALLINT  # exact zero sums too (dropped entries)
    n_cols = 300
    rp, ci, v = orc.gen_csr(40 + rows + k, rows, n_cols, kind=orc.ROWLEN_UNIFORM, a=0, b=9, value_kind=vk, dtype=dt)
    a = Csr.from_csr_arrays((rows, n_cols), rp, ci, v)
    x_cols = orc.gen_x_cols(41 + k, n_cols, k, value_kind=vk, dtype=dt)
    exp = oracle_mul_dense(orc, a, x_cols)
    assert_csr_bits(a.mul_dense(Dense.from_columns(x_cols)), *exp)

    lib = _lib.load()
    h, t = ctypes.c_void_p(), ctypes.c_void_p()
    _lib.check(lib.bsm_csr_mul_dense(a._device().handle, k, n_cols, _lib.ptr_array(x_cols), ctypes.byref(h)))
    r = _lib.DeviceCsr(h.value)
    assert r.nnz == int(exp[0][-1])
    _lib.check(lib.bsm_csr_transpose(r.handle, ctypes.byref(t)))
    trp, tci, tv = _lib.DeviceCsr(t.value).download()
    ert, ect, evt = orc.transpose(rows, k, *exp)
    assert np.array_equal(trp, ert) and np.array_equal(tci, ect)
    assert np.array_equal(tv.view(np.uint8), np.asarray(evt, dt).view(np.uint8))

    monkeypatch.setenv("BSM_SMALL_OUT", "0")
    assert_csr_bits(a.mul_dense(Dense.from_columns(x_cols)), *exp)


@pytest.mark.parametrize("variant", [1, 2, 3, 4, 5, 6])
def test_mul_dense_k32_kernel_variants(orc, monkeypatch, variant):
    """Every k = 32 f64 kernel (BSM_SPMM_VARIANT: row-wave, one row per wave
    unpipelined / x4 / x8, four rows per wave U = 4 / 2) on ragged rows with
    empty and long ones: all bit-exact."""
    monkeypatch.setenv("BSM_SPMM_VARIANT", str(variant))
    rows, n_cols, k = 901, 3000, 32
    lens = np.array([(r * 37) % 23 if r % 50 else 700 + r for r in range(rows)], dtype=np.uint64)
    lens[::7] = 0
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    ci, vals = orc.gen_entries(8, rp, n_cols)
    a = Csr.from_csr_arrays((rows, n_cols), rp, ci, vals)
    x_cols = orc.gen_x_cols(9, n_cols, k, value_kind=orc.VAL_SMALLINT)
    assert_csr_bits(a.mul_dense(Dense.from_columns(x_cols)), *oracle_mul_dense(orc, a, x_cols))


@pytest.mark.parametrize("panel", [1, 37, 350, 699])
def test_mul_dense_panelled_parity(orc, monkeypatch, panel):
    """Column-panel schedule (k = 32, f64), forced at a small size through
    BSM_SPMM_PANEL_COLS: rows cut into one slice per panel, sums carried
    through Y between passes, same bits as the oracle. Empty rows, rows
    inside one panel and rows spanning every panel included."""
    monkeypatch.setenv("BSM_SPMM_PANEL_COLS", str(panel))
    rows, n_cols, k = 1500, 700, 32
    rp, ci, v = orc.gen_csr(70 + panel, rows, n_cols, kind=orc.ROWLEN_UNIFORM, a=0, b=90)
    a = Csr.from_csr_arrays((rows, n_cols), rp, ci, v)
    x_cols = orc.gen_x_cols(71, n_cols, k, value_kind=orc.VAL_SMALLINT)  # exact zeros too
    got = a.mul_dense(Dense.from_columns(x_cols))
    assert_csr_bits(got, *oracle_mul_dense(orc, a, x_cols))
    assert a._device().plan_width() == panel


def test_mul_dense_panel_plan_rejects_unsorted_rows(orc, monkeypatch):
    """A row whose columns go back to an earlier panel would be summed out of
    storage order by the panel schedule: the plan is refused and the one-pass
    kernel runs (still bit-exact)."""
    monkeypatch.setenv("BSM_SPMM_PANEL_COLS", "100")
    rows, n_cols, k = 300, 400, 32
    rp, ci, v = orc.gen_csr(5, rows, n_cols, kind=orc.ROWLEN_UNIFORM, a=1, b=30)
    ci = ci.copy()
    lo, hi = int(rp[7]), int(rp[8])
    ci[lo:hi] = ci[lo:hi][::-1].copy()  # row 7 descending
    a = Csr.from_csr_arrays((rows, n_cols), rp, ci, v)
    x_cols = orc.gen_x_cols(6, n_cols, k)
    got = a.mul_dense(Dense.from_columns(x_cols))
    assert_csr_bits(got, *oracle_mul_dense(orc, a, x_cols))
    assert a._device().plan_width() == 0


@pytest.mark.parametrize("dtype", [np.float64, np.float32, np.int64])
def test_mul_dense_exact_cancellations(orc, dtype):
    """Small-integer values and an X with ~1/7 zeros: exact sums that hit 0
    must be dropped exactly as insert does (sparse.rs:229)."""
    dt = np.dtype(dtype)
    rows, n_cols, k = 2000, 50, 5
    rp, ci, v = orc.gen_csr(3, rows, n_cols, kind=orc.ROWLEN_UNIFORM, a=0, b=12, value_kind=orc.VAL_SMALLINT,
                            dtype=dt)
    a = Csr.from_csr_arrays((rows, n_cols), rp, ci, v)
    x_cols = orc.gen_x_cols(4, n_cols, k, value_kind=orc.VAL_SMALLINT, dtype=dt)
    got = a.mul_dense(Dense.from_columns(x_cols))
    erp, eci, ev = oracle_mul_dense(orc, a, x_cols)
    assert int(erp[-1]) < rows * k, "test must exercise zero-dropping"
    assert_csr_bits(got, erp, eci, ev)


@pytest.mark.parametrize("k,items", [(1, 2), (1, 4), (1, 8), (3, 4), (32, 4)])
def test_long_rows_and_empty_rows(orc, monkeypatch, k, items):
    """Rows longer than the SpMV LDS chunk (256*items entries, twice that in
    LDS), mixed with empty rows."""
    monkeypatch.setenv("BSM_SPMV_ITEMS", str(items))
    rows, n_cols = 40, 6000
    lens = np.array([0, 5000, 0, 3, 2100, 1, 0, 1025] + [7] * 32, dtype=np.uint64)
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    ci, vals = orc.gen_entries(5, rp, n_cols)
    a = Csr.from_csr_arrays((rows, n_cols), rp, ci, vals)
    x_cols = orc.gen_x_cols(6, n_cols, k)
    assert_csr_bits(a.mul_dense(Dense.from_columns(x_cols)), *oracle_mul_dense(orc, a, x_cols))


def test_empty_shapes(orc):
    # no rows: Csr::new((0, 5)).finalise() panics in the reference ("big eek",
    # sparse.rs:209-211: row_index [0] is longer than 0 rows)
    with pytest.raises(Panic):
        Csr.new((0, 5), np.float64).finalise()
    a = Csr.from_csr_arrays((0, 5), np.zeros(1, np.uint64), np.zeros(0, np.uint64), np.zeros(0))
    out = a.mul_dense(Dense.new_default_with_dims(3, 5))
    assert out.dims.as_tuple() == (0, 3) and list(out.row_index) == [0]
    # no entries
    a = Csr.new((4, 5), np.float64).finalise()
    out = a.mul_dense(Dense.from_columns([np.ones(5)] * 2))
    assert list(out.row_index) == [0, 0, 0, 0, 0] and out.get_nnz() == 0
    # no RHS columns
    a = Csr.from_data([[1.0, 2.0], [0.0, 3.0]])
    out = a.mul_dense(Dense(0, 2, []))
    assert out.dims.as_tuple() == (2, 0) and list(out.row_index) == [0, 0, 0]


def test_bench_like_running_max_u32_wrapping(orc):
    """The reference bench builds A with random (row, col) inserts
    (benches/sparse_dense_mul.rs:17-22): insert_unchecked assigns entries to
    the running-max row, leaving a few huge rows with unsorted, duplicated
    columns; u32 sums wrap (Cargo.toml:18). rand's StdRng is not vendored,
    so the inputs are synthetic draws of the same shape."""
    rng = np.random.default_rng(1000)
    a = Csr.new((1000, 1000), np.uint32)
    e = 20000
    rws = rng.integers(0, 1000, e)
    cls = rng.integers(0, 1000, e)
    vs = rng.integers(0, 255, e)
    for r, c, v in zip(rws, cls, vs):
        a.insert(int(v) * 2_000_000, int(r), int(c))  # large values: force wrap-around
    a = a.finalise()
    x = Dense.new_default_with_dims(10, 1000, dtype=np.uint32)
    for _ in range(e // 100):
        x.get_col_mut(int(rng.integers(0, 10)))[int(rng.integers(0, 1000))] = int(rng.integers(0, 255)) * 3_000
    got = a.mul_dense(x)
    rp, ci, v = orc.mul_dense(1000, 1000, a.row_index, a.col_index, a.v, [x.get_col(j) for j in range(10)])
    assert_csr_bits(got, rp, ci, v)
    lens = np.diff(np.asarray(a.row_index, dtype=np.int64))
    assert lens.max() > e // 2  # the skew the reference's bench really has


def test_unfinalised_matrix_mul_dense(orc):
    a = Csr.new((3, 3), np.float64)
    a.insert(1.0, 0, 0)
    a.insert(2.0, 2, 1)  # row_index = [0, 1, 1]: all rows registered
    x = [np.array([1.0, 2.0, 3.0])]
    got = a.mul_dense(Dense.from_columns(x))
    rp, ci, v = orc.mul_dense(3, 3, a.row_index, a.col_index, a.v, x)
    assert_csr_bits(got, rp, ci, v)
    b = Csr.new((3, 3), np.float64)
    b.insert(1.0, 0, 0)  # row_index = [0]: row 1 out of bounds
    with pytest.raises(Panic):
        b.mul_dense(Dense.from_columns(x))


def test_nan_kept_inf(orc):
    a = Csr.from_data([[1.0, 0.0], [np.inf, 1.0], [0.0, 2.0]])
    x = [np.array([0.0, 1.0]), np.array([np.nan, 0.0])]
    got = a.mul_dense(Dense.from_columns(x))
    rp, ci, v = orc.mul_dense(3, 2, a.row_index, a.col_index, a.v, x)
    assert list(got.row_index) == list(rp) and list(got.col_index) == list(ci)
    assert np.array_equal(np.asarray(got.v), v, equal_nan=True)


# ------------------------------------------------------------- mul_vector
@pytest.mark.parametrize("dtype", [np.float64, np.float32, np.int32, np.uint64])
def test_mul_vector_random(orc, dtype):
    dt = np.dtype(dtype)
    vk = orc.VAL_UNIFORM if dt.kind == "f" else orc.VAL_SMALLINT
    rows, n_cols = 3000, 900
    rp, ci, v = orc.gen_csr(21, rows, n_cols, kind=orc.ROWLEN_UNIFORM, a=0, b=30, value_kind=vk, dtype=dt)
    a = Csr.from_csr_arrays((rows, n_cols), rp, ci, v)
    x = orc.gen_x_cols(22, n_cols, 1, value_kind=vk, dtype=dt)[0]
    exp = orc.mul_vector(rows, n_cols, rp, ci, v, x)
    ib = {8: np.uint64, 4: np.uint32}[dt.itemsize]
    for items in ("2", "4", "8"):  # SpMV chunk sizes
        with pytest.MonkeyPatch.context() as mp:
            mp.setenv("BSM_SPMV_ITEMS", items)
            out = np.zeros(rows, dtype=dt)
            a.mul_vector(x, out)
        assert np.array_equal(out.view(ib), exp.view(ib))  # includes -0.0 of empty rows


def test_mul_vector_unsorted_duplicates(orc):
    """Unsorted and duplicated columns: the reference sums in ascending
    column order (it walks the transpose), not storage order."""
    a = Csr.new((3, 4), np.float64)
    for val, r, c in [(1e16, 0, 3), (1.0, 0, 0), (-1e16, 0, 1), (3.0, 1, 2), (0.5, 1, 2), (2.0, 1, 0),
                      (1.0, 2, 1)]:
        a.insert(val, r, c)
    a = a.finalise()
    x = np.array([1.0, 1.0, 1.0, 1.0])
    out = np.zeros(3)
    a.mul_vector(x, out)
    exp = orc.mul_vector(3, 4, a.row_index, a.col_index, a.v, x)
    assert out.view(np.uint64).tolist() == exp.view(np.uint64).tolist()


# ------------------------------------------------------------- transpose
@pytest.mark.parametrize("dtype", [np.float64, np.int32])
def test_transpose_random(orc, dtype):
    dt = np.dtype(dtype)
    vk = orc.VAL_UNIFORM if dt.kind == "f" else orc.VAL_SMALLINT
    rows, n_cols = 2500, 3100
    rp, ci, v = orc.gen_csr(31, rows, n_cols, kind=orc.ROWLEN_UNIFORM, a=0, b=50, value_kind=vk, dtype=dt)
    a = Csr.from_csr_arrays((rows, n_cols), rp, ci, v)
    t = a.transpose()
    assert t.dims.as_tuple() == (n_cols, rows)
    assert_csr_bits(t, *orc.transpose(rows, n_cols, rp, ci, v))


def test_transpose_duplicates_stable(orc):
    a = Csr.new((3, 3), np.int32)
    for val, r, c in [(1, 0, 2), (2, 0, 2), (3, 1, 0), (4, 2, 2), (5, 2, 0)]:
        a.insert(val, r, c)
    a = a.finalise()
    assert_csr_bits(a.transpose(), *orc.transpose(3, 3, a.row_index, a.col_index, a.v))
