"""Multi-GPU Csr::mul_dense through the C-ABI (include/bsm.h, "multi-GPU").

BASELINE.json north_star: the CSR is row-block partitioned across the GPUs of
one node, the dense RHS replicated, and the dense result assembled by an RCCL
all-gather over xGMI. The partition, the per-device SpMMs, the all-gathers
(libbsm_hip.so's own RCCL communicators) and the compaction all live behind
the C-ABI (csrc/multi.hip), where a Rust ``mul_dense`` reaches them too
(INTEGRATION.md). This module is the ctypes mirror:

* :class:`MultiGpu` -- ``bsm_multi_create(n_gpus)`` (one process, n devices,
  ``ncclCommInitAll``) or, one process per GPU, ``MultiGpu.for_rank(id, world,
  rank, device)`` (``ncclCommInitRank``; rank 0 makes the id with
  :func:`unique_id` and the caller ships it), or, with the caller's own
  transport, ``MultiGpu.external(world, rank, device)`` (no communicator:
  ``step`` runs this rank's rounds into its slots, the caller exchanges the
  slots, e.g. :func:`basic_sparse_matrix_amd.distributed.exchange_slots` over
  any torch.distributed backend, then ``compact``).
* :class:`MultiCsr` -- a matrix partitioned over a context:
  ``upload`` (host arrays) or ``generate`` (bsm_synth.h, on each device),
  ``mul_dense_cols`` (host columns in, a device Csr out), and the device-level
  ``step`` / ``sync`` / ``step_times`` that bench.py times.

There is no CPU fallback: without the library or a device every call raises.
"""

from __future__ import annotations

import ctypes
import os

import numpy as np

from . import _lib

SCHEDULES = {"auto": 0, "tiled": 1, "panel": 2}
PLAN_KEYS = ("total", "tiled_count", "tiled_scan", "tiled_alloc", "tiled_write", "panel_plans", "buffers")


def partition_rows(row_ptr, pieces: int) -> np.ndarray:
    """bsm_partition_rows: the piece bounds the library uses (host only)."""
    rp = np.ascontiguousarray(row_ptr, dtype=np.uint64)
    if rp.size == 0:  # row_ptr holds rows + 1 entries: empty is not a matrix (rows would wrap to 2^64 - 1)
        raise ValueError("partition_rows: row_ptr must hold rows + 1 entries, got an empty array")
    out = np.empty(pieces + 1, dtype=np.uint64)
    _lib.check(_lib.load().bsm_partition_rows(_lib.ptr(rp), rp.size - 1, pieces, _lib.ptr(out)))
    return out


def unique_id() -> bytes:
    """bsm_multi_unique_id: the RCCL id rank 0 ships to every rank."""
    lib = _lib.require_device()
    buf = ctypes.create_string_buffer(_lib.BSM_UNIQUE_ID_BYTES)
    _lib.check(lib.bsm_multi_unique_id(buf))
    return buf.raw


class MultiGpu:
    """Owner of a bsm_multi context (SURVEY.md §8b bsm_init / bsm_finalize)."""

    def __init__(self, n_gpus: int = 1, devices=None, _handle: int | None = None):
        lib = _lib.require_device()
        if _handle is None:
            h = ctypes.c_void_p()
            devs = None
            if devices is not None:
                devs = (ctypes.c_int * len(devices))(*devices)
            _lib.check(lib.bsm_multi_create(n_gpus, devs, ctypes.byref(h)))
            _handle = h.value
        self.handle = _handle
        w, n, r = ctypes.c_int(), ctypes.c_int(), ctypes.c_int()
        _lib.check(lib.bsm_multi_info(self.handle, ctypes.byref(w), ctypes.byref(n), ctypes.byref(r)))
        self.world, self.n_local, self.first_rank = w.value, n.value, r.value

    @classmethod
    def for_rank(cls, uid: bytes, world: int, rank: int, device: int) -> "MultiGpu":
        lib = _lib.require_device()
        if len(uid) != _lib.BSM_UNIQUE_ID_BYTES:
            raise ValueError("unique id must be BSM_UNIQUE_ID_BYTES long")
        h = ctypes.c_void_p()
        buf = ctypes.create_string_buffer(uid, _lib.BSM_UNIQUE_ID_BYTES)
        _lib.check(lib.bsm_multi_create_rank(buf, world, rank, device, ctypes.byref(h)))
        return cls(_handle=h.value)

    @classmethod
    def external(cls, world: int, rank: int, device: int) -> "MultiGpu":
        """bsm_multi_create_external: rank `rank` of `world` on `device`, no
        RCCL communicator (the slots of the gathered Y move by the caller's
        transport)."""
        lib = _lib.require_device()
        h = ctypes.c_void_p()
        _lib.check(lib.bsm_multi_create_external(world, rank, device, ctypes.byref(h)))
        return cls(_handle=h.value)

    @property
    def is_external(self) -> bool:
        e = ctypes.c_int(0)
        _lib.check(_lib.load().bsm_multi_is_external(self.handle, ctypes.byref(e)))
        return bool(e.value)

    def broadcast(self, ptrs, nbytes: int, root: int = 0) -> None:
        """ncclBroadcast of `nbytes` from global rank `root` into ptrs[i] on
        every local device (synchronous)."""
        _lib.check(_lib.load().bsm_multi_broadcast(self.handle, _lib.ptr_array(list(ptrs)), nbytes, root))

    def close(self) -> None:
        if getattr(self, "handle", None) and _lib._lib is not None:
            _lib._lib.bsm_multi_destroy(self.handle)
            self.handle = None

    def __del__(self):
        self.close()


class MultiCsr:
    """Owner of a bsm_mcsr: a CSR cut into chunks x world nnz-balanced row
    blocks over a context's devices. Keeps the context alive."""

    def __init__(self, ctx: MultiGpu, handle: int, dtype):
        self.ctx, self.handle, self.dtype = ctx, handle, np.dtype(dtype)
        lib = _lib.load()
        r, c, n, pr = _lib._u64(), _lib._u64(), _lib._u64(), _lib._u64()
        p = ctypes.c_uint32()
        _lib.check(lib.bsm_mcsr_info(handle, ctypes.byref(r), ctypes.byref(c), ctypes.byref(n), ctypes.byref(p),
                                     ctypes.byref(pr), None))
        self.rows, self.cols, self.nnz, self.pieces, self.piece_rows = r.value, c.value, n.value, p.value, pr.value
        self.k = None

    @classmethod
    def upload(cls, ctx: MultiGpu, rows: int, cols: int, row_ptr, col_idx, vals, chunks: int = 1) -> "MultiCsr":
        lib = _lib.require_device()
        vals = np.ascontiguousarray(vals)
        code = _lib.DTYPE_CODES.get(vals.dtype)
        if code is None:
            raise TypeError(f"dtype {vals.dtype} has no GPU path")
        rp = np.ascontiguousarray(row_ptr, dtype=np.uint64)
        ci = np.ascontiguousarray(col_idx, dtype=np.uint64)
        h = ctypes.c_void_p()
        _lib.check(lib.bsm_mcsr_upload(ctx.handle, code, rows, cols, vals.size, _lib.ptr(rp), _lib.ptr(ci),
                                       _lib.ptr(vals), chunks, ctypes.byref(h)))
        return cls(ctx, h.value, vals.dtype)

    @classmethod
    def generate(cls, ctx: MultiGpu, seed: int, rows: int, n_cols: int, rowlen_kind=_lib.ROWLEN_CONST, a=10, b=10,
                 value_kind=_lib.VAL_UNIFORM, dtype=np.float64, chunks: int = 1) -> "MultiCsr":
        lib = _lib.require_device()
        dt = np.dtype(dtype)
        h = ctypes.c_void_p()
        _lib.check(lib.bsm_mcsr_generate(ctx.handle, _lib.DTYPE_CODES[dt], seed, rows, n_cols, rowlen_kind, a, b,
                                         value_kind, chunks, ctypes.byref(h)))
        return cls(ctx, h.value, dt)

    def bounds(self) -> np.ndarray:
        out = np.empty(self.pieces + 1, dtype=np.uint64)
        _lib.check(_lib.load().bsm_mcsr_info(self.handle, None, None, None, None, None, _lib.ptr(out)))
        return out

    def prepare(self, k: int, schedule: str = "auto") -> dict:
        """Per-piece schedules + gathered-Y and output buffers for k columns;
        returns the host phase times (ms) of the slowest local device."""
        ms = (ctypes.c_double * len(PLAN_KEYS))()
        _lib.check(_lib.load().bsm_mcsr_prepare(self.handle, k, SCHEDULES[schedule], ms))
        self.k = k
        return {key: round(ms[i], 2) for i, key in enumerate(PLAN_KEYS)}

    def plan_info(self) -> dict:
        """Which schedule prepare built for this process's pieces."""
        nt, np_, b, pc = ctypes.c_int(), ctypes.c_int(), _lib._u64(), _lib._u64()
        _lib.check(_lib.load().bsm_mcsr_plan_info(self.handle, ctypes.byref(nt), ctypes.byref(np_), ctypes.byref(b),
                                                  ctypes.byref(pc)))
        return {"tiled_pieces": nt.value, "local_pieces": np_.value, "copy_bytes": b.value,
                "panel_cols": pc.value}

    def mul_dense_cols(self, cols, x_rows: int) -> "_lib.DeviceCsr":
        """bsm_mcsr_mul_dense: host columns of X -> the output Csr on the first
        local device (Csr::mul_dense on every GPU of the context)."""
        arrs = [np.ascontiguousarray(c) for c in cols]
        out = ctypes.c_void_p()
        rc = _lib.load().bsm_mcsr_mul_dense(self.handle, len(arrs), x_rows, _lib.ptr_array(arrs), ctypes.byref(out))
        if rc != _lib.BSM_OK:
            raise _lib.BsmError(rc, _lib.last_error())
        self.k = len(arrs)
        return _lib.DeviceCsr(out.value)

    def step(self, x_ptrs) -> None:
        """Device level, async: x_ptrs[i] = X (cols x k row-major) on local device i."""
        _lib.check(_lib.load().bsm_mcsr_step(self.handle, _lib.ptr_array(list(x_ptrs))))

    def sync(self) -> None:
        _lib.check(_lib.load().bsm_mcsr_sync(self.handle))

    def step_times(self, local: int = 0) -> list:
        """[{spmm, allgather_tail, compaction, total} ms] per step since the last reset."""
        lib = _lib.load()
        n = ctypes.c_int(0)
        _lib.check(lib.bsm_mcsr_step_times(self.handle, local, 0, ctypes.byref(n), None))
        ms = (ctypes.c_double * max(1, 4 * n.value))()
        _lib.check(lib.bsm_mcsr_step_times(self.handle, local, n.value, ctypes.byref(n), ms))
        return [{"spmm": ms[4 * s], "allgather_tail": ms[4 * s + 1], "compaction": ms[4 * s + 2],
                 "total": ms[4 * s + 3]} for s in range(n.value)]

    def reset_times(self) -> None:
        _lib.load().bsm_mcsr_reset_times(self.handle)

    def copy_y(self, local: int, y_ptr: int, nnz_ptr: int) -> None:
        """The assembled Y (rows x k row-major) and per-row nonzero counts on
        local device `local` into caller device buffers (0 = skip)."""
        _lib.check(_lib.load().bsm_mcsr_copy_y(self.handle, local, y_ptr, nnz_ptr))

    def set_output_rank(self, rank: int) -> None:
        """bsm_mcsr_set_output_rank: only global rank `rank` compacts the
        gathered Y into the output Csr (-1: every process). The other ranks
        keep no output buffers and skip the compaction. Call before
        prepare (it drops a prepared schedule's buffers)."""
        _lib.check(_lib.load().bsm_mcsr_set_output_rank(self.handle, int(rank)))

    def compact(self) -> None:
        """bsm_mcsr_compact: the gathered Y -> the output Csr (async; after the
        slot exchange on an external context)."""
        _lib.check(_lib.load().bsm_mcsr_compact(self.handle))

    def slot_read(self, first: int, n: int, local: int = 0):
        """Slots [first, first+n) of the gathered Y and its row counts on local
        device `local` -> host arrays ((n, piece_rows, k) values, (n,
        piece_rows) int32). Slot c*world + r is round c of rank r."""
        k = self.k or 0
        y = np.empty((n, self.piece_rows, k), dtype=self.dtype)
        nz = np.empty((n, self.piece_rows), dtype=np.int32)
        _lib.check(_lib.load().bsm_mcsr_slot_read(self.handle, local, first, n, _lib.ptr(y), _lib.ptr(nz)))
        return y, nz

    def slot_write(self, first: int, y, nz, local: int = 0) -> None:
        """Host arrays shaped as slot_read's -> slots [first, first+len(y))."""
        y = np.ascontiguousarray(y, dtype=self.dtype)
        nz = np.ascontiguousarray(nz, dtype=np.int32)
        n = y.shape[0]
        if y.shape[1:] != (self.piece_rows, self.k or 0) or nz.shape != (n, self.piece_rows):
            raise ValueError("slot arrays must be (n, piece_rows, k) and (n, piece_rows)")
        _lib.check(_lib.load().bsm_mcsr_slot_write(self.handle, local, first, n, _lib.ptr(y), _lib.ptr(nz)))

    def output(self) -> "_lib.DeviceCsr":
        out = ctypes.c_void_p()
        _lib.check(_lib.load().bsm_mcsr_output(self.handle, ctypes.byref(out)))
        return _lib.DeviceCsr(out.value)

    def close(self) -> None:
        if getattr(self, "handle", None) and _lib._lib is not None:
            _lib._lib.bsm_mcsr_free(self.handle)
            self.handle = None

    def __del__(self):
        self.close()


# ---------------------------------------------------------------------------
# process-wide GPU count of the host mirror's Csr.mul_dense (the Rust binding's
# OnceLock context): None = the single-GPU path
# (bsm_csr_mul_dense); n >= 1 = the row-block path on n GPUs through RCCL
# (n = 1 included, so the RCCL leg is exercised on one GPU).
_gpus: int | None = None
_ctx: MultiGpu | None = None


def set_gpus(n: int | None, chunks: int = 1) -> None:
    """Route the mirror's Csr.mul_dense over n GPUs (None: one GPU, no RCCL).
    The environment variable BSM_N_GPUS sets the same at import."""
    global _gpus, _ctx, _chunks
    if n is not None and n < 1:
        raise ValueError("n must be >= 1")
    if n != _gpus:
        _ctx = None
    _gpus, _chunks = n, max(1, int(chunks))


_chunks = 1


def gpus() -> int | None:
    return _gpus


def context() -> MultiGpu:
    global _ctx
    if _gpus is None:
        raise RuntimeError("multi-GPU mul_dense is not enabled (set_gpus)")
    if _ctx is None:
        _ctx = MultiGpu(_gpus)
    return _ctx


def chunks() -> int:
    return _chunks


if os.environ.get("BSM_N_GPUS"):
    set_gpus(int(os.environ["BSM_N_GPUS"]), int(os.environ.get("BSM_CHUNKS", "1")))
