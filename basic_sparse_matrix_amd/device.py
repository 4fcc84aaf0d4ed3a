"""Device-level (HBM-resident) entry points for benchmarks and multi-GPU runs.

Thin wrappers over the ``bsm_dev_*`` functions of include/bsm.h. PyTorch is
used only as plumbing: it allocates HBM buffers (``torch.empty(...,
device="cuda")``), supplies the HIP stream (``torch.cuda.current_stream()``)
and, in bench.py, ``torch.distributed`` (RCCL). All compute is the HIP
kernels of libbsm_hip.so.
"""

from __future__ import annotations

import ctypes
from dataclasses import dataclass

import numpy as np
import torch

from . import _lib

TORCH_DT = {
    np.dtype(np.float64): torch.float64,
    np.dtype(np.float32): torch.float32,
    np.dtype(np.int32): torch.int32,
    np.dtype(np.uint32): torch.uint32,
    np.dtype(np.int64): torch.int64,
    np.dtype(np.uint64): torch.uint64,
}


def _stream(stream=None) -> int:
    s = stream if stream is not None else torch.cuda.current_stream()
    return s.cuda_stream


def _p(t: torch.Tensor) -> int:
    return t.data_ptr() if t.numel() else 0


@dataclass
class DeviceCsrBlock:
    """A CSR row block resident in HBM: rows [row0, row0+rows) of a matrix
    with n_cols columns. row_ptr is local (starts at 0)."""

    row0: int
    rows: int
    n_cols: int
    row_ptr: torch.Tensor  # int64 [rows+1]
    col: torch.Tensor  # int32 [nnz]
    vals: torch.Tensor  # T [nnz]
    dtype: np.dtype
    panel_cols: int = 0  # column-panel plan (bsm_dev_spmm_plan), 0 = none
    seg: torch.Tensor | None = None
    tiled: "TiledPlan | None" = None  # row-block x column-panel copy (bsm_dev_tiled_create)

    @property
    def nnz(self) -> int:
        return int(self.col.numel())

    @classmethod
    def generate(cls, seed, row0, rows, n_cols, rowlen_kind=_lib.ROWLEN_CONST, a=10, b=10,
                 value_kind=_lib.VAL_UNIFORM, dtype=np.float64, device="cuda") -> "DeviceCsrBlock":
        """Synthetic CSR rows (bsm_synth.h recipe) generated on the device."""
        lib = _lib.require_device()
        dt = np.dtype(dtype)
        rp = torch.empty(rows + 1, dtype=torch.int64, device=device)
        wsb = lib.bsm_dev_scan_workspace_bytes(rows)
        ws = torch.empty(max(16, wsb), dtype=torch.uint8, device=device)
        s = _stream()
        _lib.check(lib.bsm_dev_gen_row_ptr(seed, row0, rows, n_cols, rowlen_kind, a, b, _p(rp), _p(ws), wsb, s))
        nnz = int(rp[rows].item()) if rows else 0
        col = torch.empty(nnz, dtype=torch.int32, device=device)
        vals = torch.empty(nnz, dtype=TORCH_DT[dt], device=device)
        _lib.check(lib.bsm_dev_gen_entries(_lib.DTYPE_CODES[dt], seed, row0, rows, n_cols, value_kind, _p(rp),
                                           _p(col), _p(vals), s))
        return cls(row0, rows, n_cols, rp, col, vals, dt)

    def plan(self, k: int, panel_cols: int | None = None) -> int:
        """Build the column-panel plan for k right-hand columns (synchronous,
        once per matrix). Returns the panel width in use (0 = single pass)."""
        lib = _lib.require_device()
        w = lib.bsm_dev_spmm_panel_cols(_lib.DTYPE_CODES[self.dtype], self.n_cols, k) if panel_cols is None \
            else panel_cols
        self.panel_cols, self.seg = 0, None
        nbytes = lib.bsm_dev_spmm_plan_bytes(self.rows, self.n_cols, w)
        if w == 0 or nbytes == 0:
            return 0
        seg = torch.empty(nbytes // 4, dtype=torch.int32, device=self.col.device)
        usable = ctypes.c_int(0)
        _lib.check(lib.bsm_dev_spmm_plan(self.rows, self.n_cols, _p(self.row_ptr), _p(self.col), w, _p(seg),
                                         ctypes.byref(usable), _stream()))
        if usable.value:
            self.panel_cols, self.seg = w, seg
        return self.panel_cols

    def plan_tiled(self, k: int, force: bool = False) -> "TiledPlan | None":
        """Build the row-block x column-panel copy for k right-hand columns
        when the library wants it for this shape (f64; k = 32 and X > 1 GiB, or
        k = 1 and X > 4 MiB), or
        whenever possible with force (any chunk padding accepted). Synchronous, once per matrix. Returns
        the plan, or None (shape not served, or no memory for the copy)."""
        lib = _lib.require_device()
        self.tiled = None
        if self.dtype != np.float64 or k not in (1, 32) or self.nnz == 0:
            return None
        if not force:
            max_len = int((self.row_ptr[1:] - self.row_ptr[:-1]).max().item()) if self.rows else 0
            if not lib.bsm_dev_tiled_wanted(_lib.DTYPE_CODES[self.dtype], self.rows, self.n_cols, self.nnz, k,
                                            max_len):
                return None
        h = ctypes.c_void_p()
        rc = lib.bsm_dev_tiled_create(self.rows, self.n_cols, self.nnz, _p(self.row_ptr), _p(self.col),
                                      _p(self.vals), k, _lib.BSM_TILED_ANY_PADDING if force else 0,
                                      ctypes.byref(h), _stream())
        if rc in (_lib.BSM_ERR_UNSUPPORTED, _lib.BSM_ERR_OOM):
            return None
        _lib.check(rc)
        self.tiled = TiledPlan(h.value, k)
        return self.tiled

    def spmm(self, x: torch.Tensor, y: torch.Tensor, row_nnz: torch.Tensor | None = None, stream=None) -> None:
        """Y = A X (x: n_cols x k row-major, y: rows x k row-major), async.
        Uses the tiled copy or the column-panel plan when one was built (same
        bits)."""
        lib = _lib.load()
        k = x.shape[1] if x.dim() == 2 else 1
        if self.tiled is not None and k == self.tiled.k:
            _lib.check(lib.bsm_dev_spmm_tiled(self.tiled.handle, _p(x), _p(y),
                                              _p(row_nnz) if row_nnz is not None else 0, _stream(stream)))
            return
        if self.seg is not None:
            _lib.check(lib.bsm_dev_spmm_panelled(_lib.DTYPE_CODES[self.dtype], self.rows, self.n_cols, self.nnz,
                                                 _p(self.row_ptr), _p(self.col), _p(self.vals), k, _p(x), _p(y),
                                                 _p(row_nnz) if row_nnz is not None else 0, self.panel_cols,
                                                 _p(self.seg), _stream(stream)))
            return
        _lib.check(lib.bsm_dev_spmm(_lib.DTYPE_CODES[self.dtype], self.rows, self.n_cols, self.nnz, _p(self.row_ptr),
                                    _p(self.col), _p(self.vals), k, _p(x), _p(y),
                                    _p(row_nnz) if row_nnz is not None else 0, _stream(stream)))


class TiledPlan:
    """Owner of a bsm_tiled handle (the row-block x column-panel copy)."""

    def __init__(self, handle: int, k: int = 32):
        self.handle = handle
        self.k = k

    def info(self) -> dict:
        lib = _lib.load()
        b, sl, pc = ctypes.c_uint64(), ctypes.c_uint64(), ctypes.c_uint64()
        _lib.check(lib.bsm_tiled_info(self.handle, ctypes.byref(b), ctypes.byref(sl), ctypes.byref(pc)))
        return {"bytes": b.value, "slots": sl.value, "panel_cols": pc.value}

    def __del__(self):
        if getattr(self, "handle", None) and _lib._lib is not None:
            _lib._lib.bsm_tiled_destroy(self.handle)
            self.handle = None


def gen_dense(seed, row0, n, k, value_kind=_lib.VAL_UNIFORM, dtype=np.float64, device="cuda") -> torch.Tensor:
    """Row-major n x k dense operand X[r][j] = bsm_x_value(seed, row0+r, j)."""
    lib = _lib.require_device()
    dt = np.dtype(dtype)
    x = torch.empty((n, k), dtype=TORCH_DT[dt], device=device)
    _lib.check(lib.bsm_dev_gen_dense(_lib.DTYPE_CODES[dt], seed, row0, n, k, value_kind, _p(x), _stream()))
    return x


class Compactor:
    """Dense Y -> output Csr (the zero-dropping insert of sparse.rs:229) with
    preallocated worst-case buffers, so a timed step allocates nothing."""

    def __init__(self, rows: int, k: int, dtype, device="cuda"):
        lib = _lib.load()
        self.rows, self.k, self.dtype = rows, k, np.dtype(dtype)
        self.row_ptr = torch.empty(rows + 1, dtype=torch.int64, device=device)
        self.col = torch.empty(max(1, rows * k), dtype=torch.int32, device=device)
        self.vals = torch.empty(max(1, rows * k), dtype=TORCH_DT[self.dtype], device=device)
        self.ws_bytes = lib.bsm_dev_scan_workspace_bytes(rows)
        self.ws = torch.empty(max(16, self.ws_bytes), dtype=torch.uint8, device=device)

    def __call__(self, y: torch.Tensor, row_nnz: torch.Tensor, stream=None) -> None:
        lib = _lib.load()
        _lib.check(lib.bsm_dev_compact(_lib.DTYPE_CODES[self.dtype], self.rows, self.k, _p(y), _p(row_nnz),
                                       _p(self.row_ptr), _p(self.col), _p(self.vals), _p(self.ws), self.ws_bytes,
                                       _stream(stream)))

    def nnz(self) -> int:
        return int(self.row_ptr[self.rows].item())


def gen_insert_stream(seed, n, rows=1000, cols=1000, vmod=255, dtype=np.uint32, device="cuda"):
    """Bench-shaped insert stream on the device (bsm_dev_gen_insert_stream;
    benches/sparse_dense_mul.rs:16-22): (row u64, col u64, v dtype) tensors."""
    lib = _lib.require_device()
    dt = np.dtype(dtype)
    r = torch.empty(max(1, n), dtype=torch.uint64, device=device)
    c = torch.empty(max(1, n), dtype=torch.uint64, device=device)
    v = torch.empty(max(1, n), dtype=TORCH_DT[dt], device=device)
    _lib.check(lib.bsm_dev_gen_insert_stream(_lib.DTYPE_CODES[dt], seed, 0, n, rows, cols, vmod, _p(r), _p(c), _p(v),
                                             _stream()))
    return r[:n], c[:n], v[:n]


def csr_from_device_inserts(dims, row: torch.Tensor, col: torch.Tensor, v: torch.Tensor, stream=None):
    """bsm_dev_csr_from_inserts on device tensors -> a finalised host Csr
    whose device copy stays cached (Csr::insert x n, then finalise)."""
    from .sparse import Csr, _raise_for
    from .util import MatDim

    lib = _lib.require_device()
    d = MatDim.of(dims)
    dt = np.dtype(str(v.dtype).replace("torch.", ""))
    h = ctypes.c_void_p()
    rc = lib.bsm_dev_csr_from_inserts(_lib.DTYPE_CODES[dt], d.rows, d.cols, v.numel(), _p(row), _p(col), _p(v),
                                      ctypes.byref(h), _stream(stream))
    _raise_for(rc)
    return Csr._from_device(_lib.DeviceCsr(h.value))
