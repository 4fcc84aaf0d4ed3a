"""Where the public download's time goes (bsm_csr_download into fresh numpy
arrays): allocation, the library call (BSM_XFER_DEBUG=1 prints its DMA
phases), and freeing the previous result."""
import sys
import time

import numpy as np
import torch

sys.path.insert(0, ".")
from basic_sparse_matrix_amd import _lib  # noqa: E402
from basic_sparse_matrix_amd.device import DeviceCsrBlock  # noqa: E402

dev = torch.device("cuda", 0)
blk = DeviceCsrBlock.generate(1000, 0, 4_000_000, 1_000_000, 0, 8, 8, 0, np.float64, device=dev)
d = _lib.DeviceCsr.upload(4_000_000, 1_000_000, blk.row_ptr.cpu().numpy().astype(np.uint64),
                          blk.col.cpu().numpy().astype(np.uint64), blk.vals.cpu().numpy())
lib = _lib.load()
for i in range(4):
    t0 = time.perf_counter()
    rp = np.empty(d.rows + 1, np.uint64)
    ci = np.empty(d.nnz, np.uint64)
    v = np.empty(d.nnz, np.float64)
    t1 = time.perf_counter()
    _lib.check(lib.bsm_csr_download(d.handle, _lib.ptr(rp), _lib.ptr(ci), _lib.ptr(v)))
    t2 = time.perf_counter()
    del rp, ci, v
    t3 = time.perf_counter()
    print(f"alloc {1e3 * (t1 - t0):.2f} ms, download {1e3 * (t2 - t1):.2f} ms, free {1e3 * (t3 - t2):.2f} ms", flush=True)
