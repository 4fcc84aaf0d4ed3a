"""Recycled host pages for the arrays a GPU result is downloaded into.

A public ``Csr.mul_dense`` at C3 returns 520 MB of host arrays (usize
col_index + f64 v, as the reference's ``Csr`` holds them, sparse.rs:426-446).
Fresh arrays cost twice on the host, not on the device: their first touch
is a zero-fill fault per 4 KiB page (43-48 ms on the box), and freeing the
previous result unmaps the same pages again (25-30 ms;
``profiles/r03_f1_marshal_c3.log``). The DMA itself takes ~11 ms.

This module is the host-side counterpart of the library's device caching:
result arrays are views of anonymous mappings that are 2 MiB aligned and
advised as transparent huge pages. When the last array of a result dies, its
mapping goes back to a free list (not to the kernel), already faulted in, and
the next download of a similar size reuses it. ``BSM_HOST_POOL=0`` turns the
pool off (plain ``numpy.empty``); ``BSM_HOST_POOL_MB`` caps the bytes kept
free (default 4096).

A Rust caller gets the same effect by downloading into reused ``Vec``s
(INTEGRATION.md §2): ``bsm_csr_download`` writes into caller-owned memory.
"""
from __future__ import annotations

import ctypes
import mmap
import os
import threading
import weakref

import numpy as np

_HUGE = 2 << 20
_MIN_POOLED = 1 << 20  # below this numpy's allocator is cheap enough
_REGISTER_MAX = 1 << 30


def _register(addr: int, nbytes: int) -> bool:
    """Page-lock [addr, addr + nbytes) for direct DMA (bsm_host_register)
    when the library and a device are there; the pool works without it."""
    if os.environ.get("BSM_HOST_POOL_REGISTER", "1") == "0":
        return False
    try:
        from . import _lib

        lib = _lib.require_device()
        return lib.bsm_host_register(ctypes.c_void_p(addr), nbytes) == _lib.BSM_OK
    except Exception:  # no library / device: plain pageable pages
        return False


class _Mapping:
    __slots__ = ("mm", "base", "cap", "addr", "registered", "__weakref__")

    def __init__(self, cap: int):
        # one extra huge page so the usable range can start 2 MiB aligned
        self.mm = mmap.mmap(-1, cap + _HUGE, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
        addr = ctypes.addressof(ctypes.c_char.from_buffer(self.mm))
        self.base = (-addr) % _HUGE
        self.cap = cap
        self.addr = addr + self.base
        if hasattr(mmap, "MADV_HUGEPAGE"):
            try:
                self.mm.madvise(mmap.MADV_HUGEPAGE)
            except OSError:
                pass
        # page-locked once for the mapping's life: every download into it is
        # then one direct DMA (and its pages are faulted in here, once). Not
        # past 1 GiB: the direct path stops at 128M entries, and pinning a
        # C4-sized result (2.56 GB per array) each time the free list's cap
        # evicts it cost more than it saved (multi_api_ms 343 -> 507 ms)
        self.registered = cap <= _REGISTER_MAX and _register(self.addr, cap)
        if self.registered:
            weakref.finalize(self, _unregister, self.addr)


def _unregister(addr: int) -> None:
    try:
        from . import _lib

        if _lib._lib is not None:
            _lib._lib.bsm_host_unregister(ctypes.c_void_p(addr))
    except Exception:
        pass


class HostPool:
    """Free list of page-resident mappings, best fit by capacity."""

    def __init__(self, keep_bytes: int):
        self.keep = keep_bytes
        self._free: list[_Mapping] = []
        self._free_bytes = 0
        self._mu = threading.RLock()  # a finalizer may run inside _take (GC)
        self._busy = False
        self._pending: list[_Mapping] = []
        self.hits = 0
        self.misses = 0

    def _take(self, nbytes: int) -> _Mapping:
        cap = -(-nbytes // _HUGE) * _HUGE
        with self._mu:
            # give-backs that a finalizer (GC) runs on this thread while the
            # list is scanned are queued and applied after the removal, so the
            # chosen mapping is the one removed
            self._busy = True
            try:
                best = None
                for i, m in enumerate(self._free):
                    # reuse when it wastes at most a quarter (+ one huge page)
                    if cap <= m.cap <= cap + cap // 4 + _HUGE and (best is None or m.cap < self._free[best].cap):
                        best = i
                m = self._free.pop(best) if best is not None else None
                if m is not None:  # out of the free bytes before the queued give-backs trim to `keep`
                    self._free_bytes -= m.cap
            finally:
                self._busy = False
                pending, self._pending = self._pending, []
                for p in pending:
                    self._give_back(p)
            if m is not None:
                self.hits += 1
                return m
            self.misses += 1
        return _Mapping(cap)

    def _give_back(self, m: _Mapping) -> None:
        with self._mu:
            if self._busy:
                self._pending.append(m)
                return
            self._free.append(m)
            self._free_bytes += m.cap
            while self._free_bytes > self.keep and self._free:
                # oldest first; dropped, not closed: a mapping handed back by
                # the finalizer is still exported until its view is gone, and
                # is unmapped when the last reference goes
                old = self._free.pop(0)
                self._free_bytes -= old.cap

    def empty(self, n: int, dtype) -> np.ndarray:
        dtype = np.dtype(dtype)
        nbytes = int(n) * dtype.itemsize
        m = self._take(max(nbytes, 1))
        view = (ctypes.c_char * max(nbytes, 1)).from_buffer(m.mm, m.base)
        # the mapping returns to the free list once the view, and with it every
        # array made from it (slices included), is gone
        weakref.finalize(view, self._give_back, m)
        return np.frombuffer(view, dtype=dtype, count=int(n))

    def clear(self) -> None:
        with self._mu:
            self._free.clear()
            self._free_bytes = 0

    @property
    def free_bytes(self) -> int:
        return self._free_bytes


_pool: HostPool | None = None
_pool_mu = threading.Lock()


def pool() -> HostPool | None:
    global _pool
    if os.environ.get("BSM_HOST_POOL", "1") == "0":
        return None
    if _pool is None:
        with _pool_mu:
            if _pool is None:
                _pool = HostPool(int(os.environ.get("BSM_HOST_POOL_MB", "4096")) << 20)
    return _pool


def empty(n: int, dtype) -> np.ndarray:
    """numpy.empty(n, dtype), from the pool when the array is large."""
    dtype = np.dtype(dtype)
    p = pool()
    if p is None or int(n) * dtype.itemsize < _MIN_POOLED:
        return np.empty(int(n), dtype=dtype)
    return p.empty(n, dtype)
