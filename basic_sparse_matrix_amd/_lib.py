"""ctypes binding of libbsm_hip.so (the C-ABI declared in include/bsm.h).

The library is built in-tree (``basic_sparse_matrix_amd/lib/libbsm_hip.so``)
by ``__graft_entry__.build()``. There is deliberately NO CPU fallback: every
compute method of the host mirror calls through this module, and if the HIP
library is missing or no gfx950 device is visible the call raises
:class:`DeviceUnavailable`.

PyTorch, when importable, is imported *before* the library is loaded so that
a process using both (bench.py, multi-GPU tests) resolves one HIP runtime
(torch's bundled libamdhip64.so.7 and ROCm's share that SONAME).
"""

from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

try:  # see module docstring: one HIP runtime per process
    import torch  # noqa: F401
except Exception:  # pragma: no cover - torch is optional for the library
    torch = None

# BSM_LIB_PATH: another build of the library (A/B of two builds in one process tree)
LIB_PATH = os.environ.get("BSM_LIB_PATH") or os.path.join(os.path.dirname(os.path.abspath(__file__)), "lib",
                                                          "libbsm_hip.so")

# bsm_dtype (include/bsm.h)
BSM_F64, BSM_F32, BSM_I32, BSM_U32, BSM_I64, BSM_U64 = range(6)
DTYPE_CODES = {
    np.dtype(np.float64): BSM_F64,
    np.dtype(np.float32): BSM_F32,
    np.dtype(np.int32): BSM_I32,
    np.dtype(np.uint32): BSM_U32,
    np.dtype(np.int64): BSM_I64,
    np.dtype(np.uint64): BSM_U64,
}
CODE_DTYPES = {v: k for k, v in DTYPE_CODES.items()}

# bsm_status
BSM_OK = 0
BSM_ERR_INVALID = 1
BSM_ERR_DIMENSIONS = 2
BSM_ERR_NON_SQUARE = 3
BSM_ERR_PANIC = 4
BSM_ERR_HIP = 5
BSM_ERR_OOM = 6
BSM_ERR_UNSUPPORTED = 7
BSM_TILED_ANY_PADDING = 1
BSM_ERR_NO_DEVICE = 8
BSM_ERR_OUT_OF_BOUNDS = 9
BSM_ERR_COMM = 10
BSM_UNIQUE_ID_BYTES = 128

# generator families (bsm_synth.h)
ROWLEN_CONST, ROWLEN_UNIFORM, ROWLEN_BINOMIAL = 0, 1, 2
VAL_UNIFORM, VAL_SMALLINT = 0, 1


class DeviceUnavailable(RuntimeError):
    """The HIP library or a gfx950 device is not available (no CPU fallback)."""


class BsmError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"bsm error {code}: {msg}")
        self.code = code
        self.msg = msg


_u64 = ctypes.c_uint64
_u32 = ctypes.c_uint32
_int = ctypes.c_int
_vp = ctypes.c_void_p
_pp = ctypes.POINTER(ctypes.c_void_p)
_u64p = ctypes.POINTER(ctypes.c_uint64)

# (name, restype, argtypes) for every symbol of include/bsm.h
SIGNATURES = [
    ("bsm_api_version", _int, []),
    ("bsm_last_error", ctypes.c_char_p, []),
    ("bsm_stage_timing", _int, [_int]),
    ("bsm_stage_times", _int, [_int, ctypes.POINTER(_int), ctypes.c_char_p, ctypes.POINTER(ctypes.c_double)]),
    ("bsm_device_count", _int, [ctypes.POINTER(_int)]),
    ("bsm_set_device", _int, [_int]),
    ("bsm_csr_upload", _int, [_int, _u64, _u64, _u64, _vp, _vp, _vp, ctypes.POINTER(_vp)]),
    ("bsm_csr_from_inserts", _int, [_int, _u64, _u64, _u64, _vp, _vp, _vp, ctypes.POINTER(_vp)]),
    ("bsm_csr_from_coo", _int, [_int, _u64, _u64, _u64, _vp, _vp, _vp, ctypes.POINTER(_vp)]),
    ("bsm_csr_shape", _int, [_vp, _u64p, _u64p, _u64p, ctypes.POINTER(_int)]),
    ("bsm_csr_download", _int, [_vp, _vp, _vp, _vp]),
    ("bsm_host_register", _int, [_vp, _u64]),
    ("bsm_host_unregister", _int, [_vp]),
    ("bsm_csr_free", None, [_vp]),
    ("bsm_csr_mul_dense", _int, [_vp, _u64, _u64, _pp, ctypes.POINTER(_vp)]),
    ("bsm_csr_mul_vector", _int, [_vp, _vp, _u64, _vp, _u64]),
    ("bsm_csr_transpose", _int, [_vp, ctypes.POINTER(_vp)]),
    ("bsm_csr_add_sparse", _int, [_vp, _vp, ctypes.POINTER(_vp)]),
    ("bsm_csr_sub_sparse", _int, [_vp, _vp, ctypes.POINTER(_vp)]),
    ("bsm_csr_mul_sparse", _int, [_vp, _vp, ctypes.POINTER(_vp)]),
    ("bsm_csr_cholesky", _int, [_vp, ctypes.POINTER(_vp)]),
    ("bsm_forward_substitution", _int, [_vp, _u64, _u64, _pp, _pp]),
    ("bsm_backward_substitution", _int, [_vp, _u64, _u64, _pp, _pp]),
    ("bsm_solve", _int, [_vp, _u64, _u64, _pp, _pp]),
    ("bsm_solve_blocked", _int, [_vp, _u64, _u64, _pp, _pp]),
    ("bsm_solve_nd", _int, [_vp, _u64, _u64, _pp, _pp]),
    ("bsm_nd_analyse", _int, [_u64, _vp, _vp, _u64, _vp, _vp, _u64, _u64p, _vp, _u64, _u64p]),
    ("bsm_nd_cache_clear", _int, []),
    ("bsm_nd_cache_info", _int, [_u64p, _u64p, _u64p, _u64p]),
    ("bsm_dev_gen_row_ptr", _int, [_u64, _u64, _u64, _u32, _int, _u32, _u32, _vp, _vp, _u64, _vp]),
    ("bsm_dev_gen_entries", _int, [_int, _u64, _u64, _u64, _u32, _int, _vp, _vp, _vp, _vp]),
    ("bsm_dev_gen_dense", _int, [_int, _u64, _u64, _u64, _u64, _int, _vp, _vp]),
    ("bsm_dev_gen_insert_stream", _int, [_int, _u64, _u64, _u64, _u64, _u64, _u64, _vp, _vp, _vp, _vp]),
    ("bsm_dev_csr_from_inserts", _int, [_int, _u64, _u64, _u64, _vp, _vp, _vp, ctypes.POINTER(_vp), _vp]),
    ("bsm_dev_scan_workspace_bytes", _u64, [_u64]),
    ("bsm_dev_spmm", _int, [_int, _u64, _u64, _u64, _vp, _vp, _vp, _u64, _vp, _vp, _vp, _vp]),
    ("bsm_csr_panel_cols", _int, [_vp, _u64p]),
    ("bsm_dev_spmm_panel_cols", _u64, [_int, _u64, _u64]),
    ("bsm_dev_spmm_plan_bytes", _u64, [_u64, _u64, _u64]),
    ("bsm_dev_spmm_plan", _int, [_u64, _u64, _vp, _vp, _u64, _vp, ctypes.POINTER(_int), _vp]),
    ("bsm_dev_spmm_panelled", _int, [_int, _u64, _u64, _u64, _vp, _vp, _vp, _u64, _vp, _vp, _vp, _u64, _vp, _vp]),
    ("bsm_dev_tiled_wanted", _int, [_int, _u64, _u64, _u64, _u64, _u64]),
    ("bsm_dev_tiled_create", _int, [_u64, _u64, _u64, _vp, _vp, _vp, _u64, _int, ctypes.POINTER(_vp), _vp]),
    ("bsm_dev_spmm_tiled", _int, [_vp, _vp, _vp, _vp, _vp]),
    ("bsm_tiled_info", _int, [_vp, _u64p, _u64p, _u64p]),
    ("bsm_tiled_destroy", None, [_vp]),
    ("bsm_csr_tiled", _int, [_vp, ctypes.POINTER(_int)]),
    ("bsm_dev_compact", _int, [_int, _u64, _u64, _vp, _vp, _vp, _vp, _vp, _vp, _u64, _vp]),
    # multi-GPU (row blocks + RCCL all-gather)
    ("bsm_multi_create", _int, [_int, ctypes.POINTER(_int), ctypes.POINTER(_vp)]),
    ("bsm_multi_unique_id", _int, [_vp]),
    ("bsm_multi_create_rank", _int, [_vp, _int, _int, _int, ctypes.POINTER(_vp)]),
    ("bsm_multi_create_external", _int, [_int, _int, _int, ctypes.POINTER(_vp)]),
    ("bsm_multi_is_external", _int, [_vp, ctypes.POINTER(_int)]),
    ("bsm_partition_rows", _int, [_vp, _u64, _u32, _vp]),
    ("bsm_multi_info", _int, [_vp, ctypes.POINTER(_int), ctypes.POINTER(_int), ctypes.POINTER(_int)]),
    ("bsm_multi_broadcast", _int, [_vp, _pp, _u64, _int]),
    ("bsm_multi_destroy", None, [_vp]),
    ("bsm_mcsr_upload", _int, [_vp, _int, _u64, _u64, _u64, _vp, _vp, _vp, _u32, ctypes.POINTER(_vp)]),
    ("bsm_mcsr_generate", _int, [_vp, _int, _u64, _u64, _u32, _int, _u32, _u32, _int, _u32, ctypes.POINTER(_vp)]),
    ("bsm_mcsr_info", _int, [_vp, _u64p, _u64p, _u64p, ctypes.POINTER(_u32), _u64p, _vp]),
    ("bsm_mcsr_prepare", _int, [_vp, _u64, _int, ctypes.POINTER(ctypes.c_double)]),
    ("bsm_mcsr_plan_info", _int, [_vp, ctypes.POINTER(_int), ctypes.POINTER(_int), _u64p, _u64p]),
    ("bsm_mcsr_mul_dense", _int, [_vp, _u64, _u64, _pp, ctypes.POINTER(_vp)]),
    ("bsm_mcsr_step", _int, [_vp, _pp]),
    ("bsm_mcsr_sync", _int, [_vp]),
    ("bsm_mcsr_step_times", _int, [_vp, _int, _int, ctypes.POINTER(_int), ctypes.POINTER(ctypes.c_double)]),
    ("bsm_mcsr_reset_times", None, [_vp]),
    ("bsm_mcsr_copy_y", _int, [_vp, _int, _vp, _vp]),
    ("bsm_mcsr_output", _int, [_vp, ctypes.POINTER(_vp)]),
    ("bsm_mcsr_compact", _int, [_vp]),
    ("bsm_mcsr_set_output_rank", _int, [_vp, _int]),
    ("bsm_mcsr_slot_read", _int, [_vp, _int, _u32, _u32, _vp, _vp]),
    ("bsm_mcsr_slot_write", _int, [_vp, _int, _u32, _u32, _vp, _vp]),
    ("bsm_mcsr_free", None, [_vp]),
]

_lock = threading.Lock()
_lib = None


def load(path: str = LIB_PATH) -> ctypes.CDLL:
    """Load the C-ABI library (no device needed) and declare its signatures."""
    global _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(path):
            raise DeviceUnavailable(
                f"{path} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'`"
            )
        lib = ctypes.CDLL(path)
        for name, res, args in SIGNATURES:
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
        return lib


def stage_timing(on: bool = True) -> None:
    """Arm (or disarm) the solver's per-stage HIP-event timer (bsm_stage_timing)."""
    check(load().bsm_stage_timing(1 if on else 0))


def stage_times() -> dict:
    """{stage: device ms} of the last solve on this thread (bsm_stage_times;
    arm it first with stage_timing())."""
    lib = load()
    n = ctypes.c_int(0)
    check(lib.bsm_stage_times(0, ctypes.byref(n), None, None))
    names = ctypes.create_string_buffer(32 * max(1, n.value))
    ms = (ctypes.c_double * max(1, n.value))()
    check(lib.bsm_stage_times(n.value, ctypes.byref(n), names, ms))
    out = {}
    for i in range(n.value):
        key = names.raw[32 * i:32 * (i + 1)].split(b"\0", 1)[0].decode()
        out[key] = out.get(key, 0.0) + ms[i]
    return out


def nd_cache_info() -> dict:
    """State of solve(order="nd")'s plan cache across handles (bsm_nd_cache_info)."""
    vals = [ctypes.c_uint64(0) for _ in range(4)]
    check(load().bsm_nd_cache_info(*[ctypes.byref(v) for v in vals]))
    return dict(zip(("entries", "kept_bytes", "hits", "misses"), (v.value for v in vals)))


def nd_cache_clear() -> None:
    """Drop every cached nd plan not also held by a live handle (bsm_nd_cache_clear)."""
    check(load().bsm_nd_cache_clear())


def last_error() -> str:
    msg = load().bsm_last_error()
    return msg.decode() if msg else ""


def check(rc: int) -> None:
    if rc != BSM_OK:
        raise BsmError(rc, last_error())


_device_ok = None


def require_device() -> ctypes.CDLL:
    """Return the library, raising DeviceUnavailable when no GPU is usable."""
    global _device_ok
    lib = load()
    if _device_ok is None:
        n = _int(0)
        rc = lib.bsm_device_count(ctypes.byref(n))
        _device_ok = rc == BSM_OK and n.value > 0
    if not _device_ok:
        raise DeviceUnavailable("no HIP device visible; this path has no CPU fallback")
    return lib


def ptr(a: np.ndarray) -> int:
    return a.ctypes.data if a.size else 0


def ptr_array(arrays) -> ctypes.Array:
    arr = (ctypes.c_void_p * max(1, len(arrays)))()
    for i, a in enumerate(arrays):
        arr[i] = ptr(a) if isinstance(a, np.ndarray) else a
    return arr


class DeviceCsr:
    """Owning wrapper of a bsm_csr* handle (device-resident finalised Csr)."""

    __slots__ = ("handle", "rows", "cols", "nnz", "dtype")

    def __init__(self, handle: int):
        lib = load()
        self.handle = handle
        r, c, n, d = _u64(), _u64(), _u64(), _int()
        check(lib.bsm_csr_shape(handle, ctypes.byref(r), ctypes.byref(c), ctypes.byref(n), ctypes.byref(d)))
        self.rows, self.cols, self.nnz = r.value, c.value, n.value
        self.dtype = CODE_DTYPES[d.value]

    @classmethod
    def upload(cls, rows, cols, row_ptr: np.ndarray, col_idx: np.ndarray, vals: np.ndarray) -> "DeviceCsr":
        lib = require_device()
        code = DTYPE_CODES.get(vals.dtype)
        if code is None:
            raise TypeError(f"dtype {vals.dtype} has no GPU path")
        row_ptr = np.ascontiguousarray(row_ptr, dtype=np.uint64)
        col_idx = np.ascontiguousarray(col_idx, dtype=np.uint64)
        vals = np.ascontiguousarray(vals)
        h = _vp()
        check(lib.bsm_csr_upload(code, rows, cols, vals.size, ptr(row_ptr), ptr(col_idx), ptr(vals), ctypes.byref(h)))
        return cls(h.value)

    @classmethod
    def from_inserts(cls, rows, cols, row: np.ndarray, col: np.ndarray, vals: np.ndarray) -> "DeviceCsr":
        """bsm_csr_from_inserts: Csr::insert(vals[i], row[i], col[i]) for every i,
        then finalise (sparse.rs:206-250), built on the device."""
        lib = require_device()
        code = DTYPE_CODES.get(vals.dtype)
        if code is None:
            raise TypeError(f"dtype {vals.dtype} has no GPU path")
        row = np.ascontiguousarray(row, dtype=np.uint64)
        col = np.ascontiguousarray(col, dtype=np.uint64)
        vals = np.ascontiguousarray(vals)
        h = _vp()
        rc = lib.bsm_csr_from_inserts(code, rows, cols, vals.size, ptr(row), ptr(col), ptr(vals), ctypes.byref(h))
        if rc != BSM_OK:
            raise BsmError(rc, last_error())
        return cls(h.value)

    @classmethod
    def from_coo(cls, rows, cols, row: np.ndarray, col: np.ndarray, vals: np.ndarray) -> "DeviceCsr":
        """bsm_csr_from_coo: From<COO<T>> for Csr<T> (sparse.rs:56-66) on the device."""
        lib = require_device()
        code = DTYPE_CODES.get(vals.dtype)
        if code is None:
            raise TypeError(f"dtype {vals.dtype} has no GPU path")
        row = np.ascontiguousarray(row, dtype=np.uint64)
        col = np.ascontiguousarray(col, dtype=np.uint64)
        vals = np.ascontiguousarray(vals)
        h = _vp()
        rc = lib.bsm_csr_from_coo(code, rows, cols, vals.size, ptr(row), ptr(col), ptr(vals), ctypes.byref(h))
        if rc != BSM_OK:
            raise BsmError(rc, last_error())
        return cls(h.value)

    def download(self):
        from . import hostpool  # recycled, page-resident result arrays

        lib = load()
        rp = hostpool.empty(self.rows + 1, np.uint64)
        ci = hostpool.empty(self.nnz, np.uint64)
        v = hostpool.empty(self.nnz, self.dtype)
        check(lib.bsm_csr_download(self.handle, ptr(rp), ptr(ci), ptr(v)))
        return rp, ci, v

    def plan_width(self) -> int:
        """Column-panel width mul_dense uses on this handle (0 = one pass)."""
        w = _u64()
        check(load().bsm_csr_panel_cols(self.handle, ctypes.byref(w)))
        return w.value

    def __del__(self):
        h = getattr(self, "handle", None)
        if h and _lib is not None:
            _lib.bsm_csr_free(h)
            self.handle = None
