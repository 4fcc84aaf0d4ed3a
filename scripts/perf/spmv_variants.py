"""A/B the k = 1 SpMV kernels on C2 (1M x 1M, 10 nnz/row) in one process:
BSM_SPMV_VARIANT is read at every launch. Prints ms per variant (HIP events,
best and mean of 20) and whether y is bit-identical to the default's."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402
import torch  # noqa: E402

from basic_sparse_matrix_amd import _lib  # noqa: E402
from basic_sparse_matrix_amd.device import DeviceCsrBlock, gen_dense  # noqa: E402

rows = n_cols = 1_000_000
blk = DeviceCsrBlock.generate(1000, 0, rows, n_cols, _lib.ROWLEN_CONST, 10, 10)
x = gen_dense(1001, 0, n_cols, 1)
y = torch.empty((rows, 1), dtype=torch.float64, device="cuda")
nnz = torch.empty(rows, dtype=torch.int32, device="cuda")
ref = None
for var in (sys.argv[1:] or ["0", "2", "3", "4", "6", "1"]):
    os.environ["BSM_SPMV_VARIANT"] = var
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    ts = []
    for i in range(23):
        e0.record()
        blk.spmm(x, y, nnz)
        e1.record()
        torch.cuda.synchronize()
        if i >= 3:
            ts.append(e0.elapsed_time(e1))
    if ref is None:
        ref = y.clone()
    same = bool(torch.equal(y.view(torch.int64), ref.view(torch.int64)))
    b_alg = 8 * (rows + 1) + 12 * blk.nnz + 8 * n_cols + 8 * rows
    print(f"BSM_SPMV_VARIANT={var}: best {min(ts) * 1e3:.1f} us, mean {np.mean(ts) * 1e3:.1f} us, "
          f"B_alg {b_alg / min(ts) / 1e6:.0f} GB/s, same bits {same}", flush=True)
