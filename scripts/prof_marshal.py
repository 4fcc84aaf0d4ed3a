#!/usr/bin/env python3
"""Where the public Csr::mul_dense call spends its time at C3 (1M x 1M, 10
nnz/row, k = 32, f64; src/sparse.rs:426-446): host Dense columns in, host Csr
(usize indices) out, A cached on the device. One JSON line per measurement:
  link_*        : torch pinned / pageable copies of 256 MB (the PCIe link itself)
  upload_x      : the library's X upload alone (bsm_csr_mul_dense with k = 32
                  minus nothing: measured as mul_dense of an empty-row matrix)
  mul_dense     : bsm_csr_mul_dense (X upload + SpMM + compaction), device handle out
  download      : bsm_csr_download of that output into usize / f64 host arrays
  public_api    : Csr.mul_dense of the Python mirror end to end
Env BSM_COPY_THREADS / BSM_STAGE_CHUNK select the staging pipeline's host
threads and chunk bytes (read once per process)."""
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from basic_sparse_matrix_amd import Csr, Dense, _lib  # noqa: E402
from basic_sparse_matrix_amd.device import DeviceCsrBlock, gen_dense  # noqa: E402


def med(fn, n=10):
    fn()
    ts = []
    for _ in range(n):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return round(1e3 * float(np.median(ts)), 3)


def emit(name, ms, **kw):
    print(json.dumps({"what": name, "ms": ms, "xfer_d2h": os.environ.get("BSM_XFER_D2H", "staged"),
                      "copy_threads": os.environ.get("BSM_COPY_THREADS", "4"),
                      "stage_chunk": os.environ.get("BSM_STAGE_CHUNK", str(16 << 20)), **kw}), flush=True)


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(0)
    nb = 256_000_000
    if "--link" in sys.argv:
        h_pin = torch.empty(nb, dtype=torch.uint8).pin_memory()
        h_page = torch.empty(nb, dtype=torch.uint8)
        h_page.fill_(1)
        d = torch.empty(nb, dtype=torch.uint8, device=dev)

        def h2d(h):
            d.copy_(h, non_blocking=True)
            torch.cuda.synchronize()

        def d2h(h):
            h.copy_(d, non_blocking=True)
            torch.cuda.synchronize()

        for nm, f in (("link_h2d_pinned", lambda: h2d(h_pin)), ("link_d2h_pinned", lambda: d2h(h_pin)),
                      ("link_h2d_pageable", lambda: h2d(h_page)), ("link_d2h_pageable", lambda: d2h(h_page))):
            ms = med(f)
            emit(nm, ms, GBps=round(nb / ms / 1e6, 1))
        a = np.ones(nb // 8)
        b = np.empty_like(a)
        ms = med(lambda: np.copyto(b, a))
        emit("host_memcpy_1thread", ms, GBps=round(nb / ms / 1e6, 1))
        del h_pin, h_page, d
    rows = n_cols = 1_000_000
    k = 32
    blk = DeviceCsrBlock.generate(1000, 0, rows, n_cols, _lib.ROWLEN_CONST, 10, 10, 0, np.float64, device=dev)
    a = Csr.from_csr_arrays((rows, n_cols), blk.row_ptr.cpu().numpy().astype(np.uint64),
                            blk.col.cpu().numpy().astype(np.uint64), blk.vals.cpu().numpy())
    del blk
    x = gen_dense(1001, 0, n_cols, k, device=dev).cpu().numpy()
    cols = [np.ascontiguousarray(x[:, j]) for j in range(k)]
    xd = Dense.from_columns(cols)
    t0 = time.perf_counter()
    h = a._device()
    emit("upload_A_once", round(1e3 * (time.perf_counter() - t0), 3), nnz=int(a.get_nnz()))
    lib = _lib.load()
    ptrs = _lib.ptr_array(cols)
    outs = []

    def mul():
        out = ctypes.c_void_p()
        _lib.check(lib.bsm_csr_mul_dense(h.handle, k, n_cols, ptrs, ctypes.byref(out)))
        outs.append(_lib.DeviceCsr(out.value))
        if len(outs) > 1:
            outs.pop(0)

    emit("mul_dense_handle", med(mul))
    o = outs[-1]
    emit("download", med(lambda: o.download()), out_nnz=o.nnz)
    # the same into destination arrays whose pages are already touched: the
    # difference is the first-touch page-fault cost of fresh host arrays
    rp_t = np.ones(o.rows + 1, np.uint64)
    ci_t = np.ones(o.nnz, np.uint64)
    v_t = np.ones(o.nnz, np.float64)
    emit("download_touched", med(lambda: _lib.check(lib.bsm_csr_download(o.handle, _lib.ptr(rp_t), _lib.ptr(ci_t),
                                                                         _lib.ptr(v_t)))))
    fresh = lambda: (np.empty(o.rows + 1, np.uint64).fill(1), np.empty(o.nnz, np.uint64).fill(1),  # noqa: E731
                     np.empty(o.nnz, np.float64).fill(1))
    emit("host_first_touch_520MB", med(fresh))
    emit("public_api", med(lambda: a.mul_dense(xd), 20))


if __name__ == "__main__":
    main()
