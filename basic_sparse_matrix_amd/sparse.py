"""Csr<T> -- host-side mirror of the reference's sparse core (src/sparse.rs).

Construction and accessors are host logic with the reference's exact
semantics (zero-skipping ``insert``, running-max row assignment in
``insert_unchecked``, ``finalise`` padding, ``get_row_compact`` /
``get_row_complete`` edge cases). The hot-path methods -- ``mul_dense``,
``mul_dense_s``, ``mul_vector``, ``transpose`` and ``cholesky_decomp`` --
check dimensions exactly where the reference does and then run on the GPU
through the C-ABI (include/bsm.h). There is no CPU fallback.

A finalised Csr is immutable (``insert`` returns Err(MatrixFinalised),
sparse.rs:223-225), so its device copy is uploaded once and cached; the
cache is not part of equality (the reference's derived PartialEq compares
the seven fields of sparse.rs:68-78).
"""

from __future__ import annotations

import ctypes
from dataclasses import dataclass
from typing import Any, List, Optional

import numpy as np

from . import _lib
from . import multi as _multi
from .dense import Dense, _infer_dtype
from .dense_static import DenseS
from .util import GetDims, MatDim, MatErr, MatErrKind, Panic

GPU_DTYPES = tuple(_lib.DTYPE_CODES.keys())


@dataclass
class CsrEntry:
    """sparse.rs:80-91 (``v`` is the value, not a reference)."""

    v: Any
    col_index: int
    row_index: int

    @staticmethod
    def of(t) -> "CsrEntry":
        """``From<(T, usize, usize)>``: (v, row, col) (sparse.rs:87-91)."""
        v, row, col = t
        return CsrEntry(v=v, col_index=int(col), row_index=int(row))

    def __eq__(self, other):
        return (
            isinstance(other, CsrEntry)
            and self.v == other.v
            and self.col_index == other.col_index
            and self.row_index == other.row_index
        )


@dataclass
class COOEntry:
    """sparse.rs:7-33: (row, col, value); ordered by row, then col."""

    row: int
    col: int
    value: Any

    @staticmethod
    def of(t) -> "COOEntry":
        """``From<(usize, usize, T)>`` (sparse.rs:13-21)."""
        r, c, v = t
        return COOEntry(int(r), int(c), v)


class COO:
    """sparse.rs:35-54: an unordered entry list with a bounds-checked insert.
    ``Csr.from_coo`` is ``From<COO<T>> for Csr<T>`` (sparse.rs:56-66)."""

    __slots__ = ("entries", "dims", "dtype")

    def __init__(self, dims, capacity: int = 0, dtype=None):
        self.dims = MatDim.of(dims)
        self.entries: List[COOEntry] = []
        self.dtype = None if dtype is None else np.dtype(dtype)

    @classmethod
    def with_capacity(cls, dims, capacity: int, dtype=None) -> "COO":
        return cls(dims, capacity, dtype)

    def insert(self, entry) -> None:
        """sparse.rs:45-53: Err(OutOfBounds) unless row < rows and col < cols."""
        e = entry if isinstance(entry, COOEntry) else COOEntry.of(entry)
        if self.dims.rows <= e.row or self.dims.cols <= e.col:
            raise MatErr(MatErrKind.OutOfBounds)
        self.entries.append(e)

    def arrays(self):
        n = len(self.entries)
        row = np.fromiter((e.row for e in self.entries), dtype=np.uint64, count=n)
        col = np.fromiter((e.col for e in self.entries), dtype=np.uint64, count=n)
        dt = self.dtype if self.dtype is not None else _infer_dtype([e.value for e in self.entries] or [0.0], None)
        v = np.asarray([e.value for e in self.entries], dtype=dt)
        return row, col, v


def _raise_for(code: int) -> None:
    if code == _lib.BSM_OK:
        return
    msg = _lib.last_error()
    if code == _lib.BSM_ERR_DIMENSIONS:
        raise MatErr(MatErrKind.IncorrectDimensions)
    if code == _lib.BSM_ERR_NON_SQUARE:
        raise MatErr(MatErrKind.NonSquareMatrix)
    if code == _lib.BSM_ERR_PANIC:
        raise Panic(msg)
    if code == _lib.BSM_ERR_OUT_OF_BOUNDS:
        raise MatErr(MatErrKind.OutOfBounds)
    raise _lib.BsmError(code, msg)


class Csr(GetDims):
    __slots__ = ("dims", "dtype", "v", "col_index", "row_index", "is_finalised", "iter_v_index",
                 "iter_row_index", "_dev", "_mdev")

    # ------------------------------------------------------------------ ctor
    def __init__(self, dims, dtype=np.int32, capacity: int = 0):
        """``Csr::new_with_capacity`` (sparse.rs:121-132)."""
        self.dims = MatDim.of(dims)
        self.dtype = np.dtype(dtype)
        self.v: Any = []
        self.col_index: Any = []
        self.row_index: Any = [0]
        self.is_finalised = False
        self.iter_v_index = 0
        self.iter_row_index = 0
        self._dev = None
        self._mdev = None  # (gpus, chunks, MultiCsr) of the multi-GPU path

    @classmethod
    def new(cls, dims, dtype=np.int32) -> "Csr":
        """sparse.rs:117-119."""
        return cls(dims, dtype)

    @classmethod
    def new_with_capacity(cls, dims, capacity: int, dtype=np.int32) -> "Csr":
        return cls(dims, dtype, capacity)

    @classmethod
    def eye(cls, dims, value, dtype=None) -> "Csr":
        """sparse.rs:134-152 (insert_unchecked: a zero value IS stored)."""
        dims = MatDim.of(dims)
        if dims.cols != dims.rows:
            raise MatErr(MatErrKind.IncorrectDimensions)
        m = cls(dims, _infer_dtype([value], dtype))
        for n in range(dims.cols):
            m._insert_unchecked(value, n, n)
        return m.finalise()

    @classmethod
    def create_diagonal(cls, contents, dtype=None) -> "Csr":
        """sparse.rs:154-160."""
        n = len(contents)
        m = cls((n, n), _infer_dtype(list(contents) or [0], dtype))
        for i, v in enumerate(contents):
            m.insert(v, i, i)
        return m.finalise()

    @classmethod
    def from_data(cls, data, dtype=None) -> "Csr":
        """sparse.rs:193-203: ``data`` is a list of ROWS; zeros are skipped."""
        rows = len(data)
        cols = len(data[0])
        m = cls((rows, cols), _infer_dtype([x for row in data for x in row] or [0], dtype))
        arr = np.asarray(data, dtype=m.dtype) if rows else np.zeros((0, cols), m.dtype)
        # vectorised equivalent of the insert loop: rows ascend, cols ascend
        nzr, nzc = np.nonzero(arr != 0) if arr.dtype.kind != "f" else np.nonzero(~(arr == 0))
        m.v = arr[nzr, nzc].copy()
        m.col_index = nzc.astype(np.uint64)
        counts = np.bincount(nzr, minlength=rows) if rows else np.zeros(0, dtype=np.int64)
        # insert_unchecked registers a row only when its first entry arrives;
        # rows after the last nonempty row are added by finalise, so the
        # result is the standard row_ptr once finalised.
        m.row_index = np.concatenate([[0], np.cumsum(counts)]).astype(np.uint64)
        m.is_finalised = True
        return m

    @classmethod
    def from_csr_arrays(cls, dims, row_index, col_index, v, dtype=None) -> "Csr":
        """Bulk constructor (this build's addition, not in the reference):
        adopt an already finalised CSR (row_index of length rows+1)."""
        m = cls(dims, v.dtype if dtype is None else dtype)
        m.v = np.ascontiguousarray(v, dtype=m.dtype)
        m.col_index = np.ascontiguousarray(col_index, dtype=np.uint64)
        m.row_index = np.ascontiguousarray(row_index, dtype=np.uint64)
        if m.row_index.shape != (m.dims.rows + 1,):
            raise ValueError("row_index must have rows+1 entries")
        m.is_finalised = True
        return m

    @classmethod
    def from_inserts(cls, dims, row, col, v) -> "Csr":
        """``insert(v[i], row[i], col[i])`` for every i, then ``finalise``
        (sparse.rs:206-250), executed on the GPU (bsm_csr_from_inserts): the
        zero skip, the running-max row rule of insert_unchecked and the
        "big eek" panic behave exactly like the sequence of calls. The result
        stays cached on the device for the hot-path methods."""
        d = MatDim.of(dims)
        v = np.asarray(v)
        if v.dtype not in GPU_DTYPES:
            raise TypeError(f"Csr<{v.dtype}> has no GPU path (supported: f64 f32 i32 u32 i64 u64)")
        try:
            dev = _lib.DeviceCsr.from_inserts(d.rows, d.cols, np.asarray(row), np.asarray(col), v)
        except _lib.BsmError as e:
            _raise_for(e.code)
            raise
        return cls._from_device(dev)

    @classmethod
    def from_coo(cls, coo: "COO") -> "Csr":
        """``From<COO<T>> for Csr<T>`` (sparse.rs:56-66) on the GPU: a stable
        sort by (row, col) (Rust's sort_by is stable), then the zero-skipping
        insert sequence and finalise. The reference's per-entry println! is
        not reproduced."""
        row, col, v = coo.arrays()
        if v.dtype not in GPU_DTYPES:
            raise TypeError(f"Csr<{v.dtype}> has no GPU path (supported: f64 f32 i32 u32 i64 u64)")
        try:
            dev = _lib.DeviceCsr.from_coo(coo.dims.rows, coo.dims.cols, row, col, v)
        except _lib.BsmError as e:
            _raise_for(e.code)
            raise
        return cls._from_device(dev)

    # ------------------------------------------------------------ building
    def finalise(self) -> "Csr":
        """sparse.rs:206-219: pad row_index to rows+1 with nnz."""
        if not self.is_finalised:
            self.is_finalised = True
            ri = list(self.row_index)
            if self.dims.rows < len(ri):
                raise Panic("big eek")
            nnz = len(self.v)
            ri.extend([nnz] * (self.dims.rows - len(ri)))
            ri.append(nnz)
            self.row_index = np.asarray(ri, dtype=np.uint64)
            self.col_index = np.asarray(self.col_index, dtype=np.uint64)
            self.v = np.asarray(self.v, dtype=self.dtype)
        return self

    def insert(self, value, row: int, col: int) -> None:
        """sparse.rs:222-233. Raises MatErr(MatrixFinalised) after finalise;
        silently ignores values equal to T::default()."""
        if self.is_finalised:
            raise MatErr(MatErrKind.MatrixFinalised)
        value = self.dtype.type(value)
        if value != 0:
            self._insert_unchecked(value, row, col)

    def _insert_unchecked(self, value, row: int, col: int) -> None:
        """sparse.rs:237-250: the row is recorded only when it exceeds the
        running maximum; an entry for an earlier row is appended to the
        current last row."""
        self.v.append(self.dtype.type(value))
        self.col_index.append(int(col))
        ri = self.row_index
        if row > len(ri) - 1:
            if row > len(ri):
                ri.append(len(self.v) - 1)
                last = ri[-1]
                ri.extend([last] * (row + 1 - len(ri)))
            else:
                ri.append(len(self.v) - 1)

    insert_unchecked = _insert_unchecked

    # ------------------------------------------------------------ accessors
    def get_dims(self) -> MatDim:
        return self.dims

    def get_nnz(self) -> int:
        """sparse.rs:162-164: last row_index entry."""
        return int(self.row_index[-1]) if len(self.row_index) else 0

    def get_density(self) -> float:
        return np.float32(len(self.v)) / np.float32(self.dims.rows * self.dims.cols)

    def _row_bounds(self, index: int):
        ri = self.row_index
        if index >= len(ri):
            raise Panic(f"index out of bounds: the len is {len(ri)} but the index is {index}")
        start = int(ri[index])
        end = len(self.v) if index == len(ri) - 1 else int(ri[index + 1])
        if start > end or end > len(self.v):
            raise Panic("slice index starts after end")
        return start, end

    def get_row_compact(self, index: int) -> List[CsrEntry]:
        """sparse.rs:252-265."""
        s, e = self._row_bounds(index)
        return [CsrEntry(v=self.v[i], col_index=int(self.col_index[i]), row_index=index) for i in range(s, e)]

    def get_row_complete(self, index: int) -> Optional[list]:
        """sparse.rs:267-294 (literal expansion, including its behaviour on
        unsorted/duplicate columns)."""
        ri = self.row_index
        if len(ri) == 0 or index >= len(ri):
            return None
        start = int(ri[index])
        end = len(self.v) if len(ri) == index + 1 else int(ri[index + 1])
        zero = self.dtype.type(0)
        out = []
        prev = 0
        for i in range(start, end):
            c = int(self.col_index[i])
            if c != 0:
                out.extend([zero] * max(0, c - prev))
            prev = c + 1
            out.append(self.v[i])
        out.extend([zero] * max(0, self.dims.cols - prev))
        return out

    def get_val_at(self, at):
        """sparse.rs:170-180."""
        at = MatDim.of(at)
        s, e = int(self.row_index[at.rows]), int(self.row_index[at.rows + 1])
        for i in range(s, e):
            if int(self.col_index[i]) == at.cols:
                return self.v[i]
        return None

    def reset_iter(self) -> None:
        self.iter_row_index = 0
        self.iter_v_index = 0

    def __iter__(self):
        return self

    def __next__(self) -> CsrEntry:
        """``Iterator for Csr`` (sparse.rs:93-114)."""
        if self.iter_v_index == len(self.v):
            raise StopIteration
        while int(self.row_index[self.iter_row_index]) == self.iter_v_index:
            self.iter_row_index += 1
        e = CsrEntry(v=self.v[self.iter_v_index], col_index=int(self.col_index[self.iter_v_index]),
                     row_index=self.iter_row_index - 1)
        self.iter_v_index += 1
        return e

    # ------------------------------------------------------- device operand
    def _csr_arrays(self):
        """(row_ptr[rows+1], col_index, v) as the reference's row loop sees
        them: an unfinalised matrix whose row_index covers every row is
        usable (its last recorded row extends to nnz, sparse.rs:256-260);
        a shorter one makes ``row_index[row]`` panic."""
        rows = self.dims.rows
        ri = np.asarray(self.row_index, dtype=np.uint64)
        nnz = len(self.v)
        if len(ri) >= rows + 1:
            rp = ri[: rows + 1].copy()
            if len(ri) == rows + 1 and not self.is_finalised:
                rp[rows] = nnz
        elif len(ri) == rows:
            rp = np.concatenate([ri, np.asarray([nnz], dtype=np.uint64)])
        else:
            raise Panic(f"index out of bounds: the len is {len(ri)} but the index is {len(ri)}")
        used = int(rp[rows]) if rows else 0
        if np.any(rp[1:] < rp[:-1]) or used > nnz:
            raise Panic("slice index starts after end")
        ci = np.asarray(self.col_index, dtype=np.uint64)[:used]
        v = np.asarray(self.v, dtype=self.dtype)[:used]
        return rp, ci, v

    def _device(self) -> "_lib.DeviceCsr":
        if self._dev is not None:
            return self._dev
        if self.dtype not in GPU_DTYPES:
            raise TypeError(f"Csr<{self.dtype}> has no GPU path (supported: f64 f32 i32 u32 i64 u64)")
        rp, ci, v = self._csr_arrays()
        if ci.size and int(ci.max()) >= self.dims.cols:
            raise Panic(f"index out of bounds: column {int(ci.max())} >= {self.dims.cols}")
        dev = _lib.DeviceCsr.upload(self.dims.rows, self.dims.cols, rp, ci, v)
        if self.is_finalised:
            self._dev = dev
        return dev

    def _panic_on_short_columns(self, cols, short) -> None:
        """rhs.get_col(c)[e.col_index] (sparse.rs:437) panics at the FIRST
        out-of-range read in the reference's loop order: rows ascending, then
        RHS columns c ascending (:432), then the row's entries in storage order
        (:435). The message names that entry's index (not the
        largest index)."""
        rp, ci, _ = self._csr_arrays()
        if not ci.size:
            return
        rows_of = np.repeat(np.arange(len(rp) - 1), np.diff(rp.astype(np.int64)))
        best = None  # (row, c, entry)
        for j in short:
            bad = np.nonzero(ci >= len(cols[j]))[0]
            if bad.size:
                e = int(bad[0])  # storage order = row order: the first bad entry has the lowest row
                key = (int(rows_of[e]), j, e)
                if best is None or key[:2] < best[:2]:
                    best = key
        if best is not None:
            _, j, e = best
            raise Panic(f"index out of bounds: the len is {len(cols[j])} but the index is {int(ci[e])}")

    def _multi_device(self):
        """The matrix partitioned over the multi-GPU context (set_gpus), cached
        like the single-GPU copy for a finalised (immutable) matrix."""
        key = (_multi.gpus(), _multi.chunks())
        if self._mdev is not None and self._mdev[0] == key:
            return self._mdev[1]
        if self.dtype not in GPU_DTYPES:
            raise TypeError(f"Csr<{self.dtype}> has no GPU path (supported: f64 f32 i32 u32 i64 u64)")
        rp, ci, v = self._csr_arrays()
        if ci.size and int(ci.max()) >= self.dims.cols:
            raise Panic(f"index out of bounds: column {int(ci.max())} >= {self.dims.cols}")
        m = _multi.MultiCsr.upload(_multi.context(), self.dims.rows, self.dims.cols, rp, ci, v, chunks=key[1])
        if self.is_finalised:
            self._mdev = (key, m)
        return m

    @classmethod
    def _from_device(cls, dev: "_lib.DeviceCsr") -> "Csr":
        rp, ci, v = dev.download()
        m = cls((dev.rows, dev.cols), dev.dtype)
        m.row_index, m.col_index, m.v = rp, ci, v
        m.is_finalised = True
        m._dev = dev
        return m

    # ------------------------------------------------------------ hot path
    def mul_dense(self, rhs: Dense) -> "Csr":
        """sparse.rs:426-446: ``self * rhs`` as a new finalised Csr of dims
        (rows, rhs.cols) with zero results dropped. GPU: spmm_rowwave /
        spmv_stream + compaction (kernels_spmm.hip)."""
        if self.dims.cols != rhs.get_dims().rows:
            raise MatErr(MatErrKind.IncorrectDimensions)
        k = rhs.get_dims().cols
        cols = [rhs.get_col(j) for j in range(k)]
        return self._mul_dense_cols(cols, rhs.get_dims().rows)

    def mul_dense_s(self, rhs: DenseS) -> "Csr":
        """sparse.rs:448-466 (dimension check against ROWS, :449)."""
        if self.dims.cols != rhs.ROWS:
            raise MatErr(MatErrKind.IncorrectDimensions)
        k = rhs.get_dims().cols
        cols = [rhs.get_col(j) for j in range(k)]
        return self._mul_dense_cols(cols, rhs.ROWS)

    def _mul_dense_cols(self, cols, x_rows: int) -> "Csr":
        for c in cols:
            if c.dtype != self.dtype:
                raise TypeError(f"mul_dense: Csr<{self.dtype}> x Dense<{c.dtype}>")
        short = [j for j, c in enumerate(cols) if len(c) < x_rows]
        if short:  # host logic: the reference panics here whatever runs the sums
            self._panic_on_short_columns(cols, short)
        lib = _lib.require_device()
        arrs = []
        for c in cols:
            a = np.ascontiguousarray(c)
            if a.shape[0] < x_rows:  # never read past its end (checked above)
                a = np.concatenate([a, np.zeros(x_rows - a.shape[0], dtype=a.dtype)])
            arrs.append(np.ascontiguousarray(a[:x_rows]))
        if _multi.gpus() is not None:  # row blocks on n GPUs + RCCL all-gather (csrc/multi.hip)
            # only the partitioned copy: no whole-matrix upload to the current device
            return Csr._from_device(self._multi_device().mul_dense_cols(arrs, x_rows))
        dev = self._device()
        out = ctypes.c_void_p()
        _raise_for(lib.bsm_csr_mul_dense(dev.handle, len(arrs), x_rows, _lib.ptr_array(arrs), ctypes.byref(out)))
        return Csr._from_device(_lib.DeviceCsr(out.value))

    def mul_vector(self, rhs, out: np.ndarray) -> None:
        """sparse.rs:468-482: writes ``out`` in place (Rust ``&mut [T]``)."""
        if self.dims.cols != len(rhs) or self.dims.rows != len(out):
            raise MatErr(MatErrKind.IncorrectDimensions)
        if not isinstance(out, np.ndarray) or out.dtype != self.dtype or not out.flags.c_contiguous:
            raise TypeError(f"out must be a contiguous numpy array of {self.dtype}")
        x = np.ascontiguousarray(rhs, dtype=self.dtype)
        dev = self._device()
        lib = _lib.require_device()
        _raise_for(lib.bsm_csr_mul_vector(dev.handle, _lib.ptr(x), len(x), _lib.ptr(out), len(out)))

    def transpose(self) -> "Csr":
        """sparse.rs:296-318 (stable CSR->CSC on the GPU)."""
        if not self.is_finalised and len(self.v):
            # the reference's row search reads row_index[row+1] past the end
            # for the last recorded row of an unfinalised matrix
            raise Panic("index out of bounds (transpose of an unfinalised matrix)")
        dev = self._device()
        lib = _lib.require_device()
        out = ctypes.c_void_p()
        _raise_for(lib.bsm_csr_transpose(dev.handle, ctypes.byref(out)))
        return Csr._from_device(_lib.DeviceCsr(out.value))

    def _sparse_binary(self, rhs: "Csr", fn_name: str) -> "Csr":
        if not isinstance(rhs, Csr) or rhs.dtype != self.dtype:
            raise TypeError(f"{fn_name}: Csr<{self.dtype}> with Csr<{getattr(rhs, 'dtype', None)}>")
        a, b = self._device(), rhs._device()
        lib = _lib.require_device()
        out = ctypes.c_void_p()
        _raise_for(getattr(lib, fn_name)(a.handle, b.handle, ctypes.byref(out)))
        return Csr._from_device(_lib.DeviceCsr(out.value))

    def add_sparse(self, rhs: "Csr") -> "Csr":
        """sparse.rs:484-540 on the GPU: the reference's per-row merge in
        storage order, zero sums dropped; Err(IncorrectDimensions) when the
        dims differ (checked here first, as the reference does)."""
        if self.get_dims() != rhs.get_dims():
            raise MatErr(MatErrKind.IncorrectDimensions)
        return self._sparse_binary(rhs, "bsm_csr_add_sparse")

    def sub_sparse(self, rhs: "Csr") -> "Csr":
        """sparse.rs:542-599 (rhs-only entries become T::default() - v)."""
        if self.get_dims() != rhs.get_dims():
            raise MatErr(MatErrKind.IncorrectDimensions)
        return self._sparse_binary(rhs, "bsm_csr_sub_sparse")

    def mul_sparse(self, rhs: "Csr") -> "Csr":
        """sparse.rs:601-635 on the GPU: dims (self.rows, rhs.cols), no
        dimension check, every entry the reference's merge of a self row with
        a row of rhs.transpose()."""
        return self._sparse_binary(rhs, "bsm_csr_mul_sparse")

    def pair_with_tranpose(self):
        """sparse.rs:320-323."""
        return self, self.transpose()

    def cholesky_decomp(self) -> "Csr":
        """``impl Csr<f32>::cholesky_decomp`` (sparse.rs:682-714); f64 is this
        build's addition."""
        if self.dtype not in (np.dtype(np.float32), np.dtype(np.float64)):
            raise TypeError("cholesky_decomp is defined for Csr<f32> (and Csr<f64> here)")
        if self.dims.rows != self.dims.cols:
            raise MatErr(MatErrKind.NonSquareMatrix)
        dev = self._device()
        lib = _lib.require_device()
        out = ctypes.c_void_p()
        _raise_for(lib.bsm_csr_cholesky(dev.handle, ctypes.byref(out)))
        return Csr._from_device(_lib.DeviceCsr(out.value))

    # ---------------------------------------------------------- comparisons
    def __eq__(self, other) -> bool:
        """Derived PartialEq over the seven fields of sparse.rs:68-78."""
        if not isinstance(other, Csr):
            return NotImplemented

        def same(a, b):
            a, b = np.asarray(a), np.asarray(b)
            return a.shape == b.shape and bool(np.all(a == b))

        return (
            self.dims == other.dims
            and same(self.v, other.v)
            and same(np.asarray(self.col_index, dtype=np.uint64), np.asarray(other.col_index, dtype=np.uint64))
            and same(np.asarray(self.row_index, dtype=np.uint64), np.asarray(other.row_index, dtype=np.uint64))
            and self.is_finalised == other.is_finalised
            and self.iter_v_index == other.iter_v_index
            and self.iter_row_index == other.iter_row_index
        )

    def clone(self) -> "Csr":
        m = Csr(self.dims, self.dtype)
        for f in ("v", "col_index", "row_index"):
            val = getattr(self, f)
            setattr(m, f, val.copy() if isinstance(val, np.ndarray) else list(val))
        m.is_finalised = self.is_finalised
        m.iter_v_index, m.iter_row_index = self.iter_v_index, self.iter_row_index
        m._dev = self._dev
        m._mdev = self._mdev
        return m

    def __repr__(self) -> str:  # Debug (sparse.rs:797-805)
        return (
            f"dims:      {self.dims}\n"
            f"v:         {list(np.asarray(self.v).tolist())}\n"
            f"col_index: {[int(c) for c in self.col_index]}\n"
            f"row_index: {[int(r) for r in self.row_index]}\n"
        )

    def __str__(self) -> str:  # Display (sparse.rs:777-795)
        out = []
        for r in range(self.dims.rows):
            row = self.get_row_complete(r)
            if row is None:
                row = [self.dtype.type(0)] * self.dims.cols
            out.append("|" + "".join(f"{x!s:>5} " for x in row) + "|")
        return "\n".join(out) + ("\n" if out else "")
