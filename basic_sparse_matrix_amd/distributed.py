"""Multi-rank Csr::mul_dense with the caller's own transport
(BASELINE.json north_star row split).

The library's multi-GPU path (csrc/multi.hip, include/bsm.h "multi-GPU")
cuts the CSR into P = chunks x world row blocks ("pieces"); piece c*world + r
is computed by rank r in round c and lands in slot c*world + r of the
gathered Y, which RCCL's in-place all-gathers fill on a context with a
communicator. On an external context (``MultiGpu.external``: no
communicator) ``MultiCsr.step`` stops after this rank's rounds and
:func:`exchange_slots` moves the slots between the ranks over any
torch.distributed process group (gloo here: host buffers). Every rank then
holds exactly what the all-gathers would have left, and ``MultiCsr.compact``
builds the output Csr through the same slot / padding / row_ptr squeeze code
as the RCCL path.

:func:`partition_rows` restates the library's piece bounds
(``bsm_partition_rows``) in Python for the CPU tests.
"""

from __future__ import annotations

import numpy as np


def partition_rows(row_ptr, pieces: int) -> np.ndarray:
    """Contiguous row blocks of near-equal cost, a row costing its entries plus
    c = max(1, nnz/rows) (csrc/multi.hip partition_by_cost): bound i is the
    first row r with rows*rp[r] + r*max(nnz, rows) >= i*total/P, total =
    nnz*rows + rows*max(nnz, rows). Exact integers (Python ints)."""
    rp = [int(v) for v in np.asarray(row_ptr, dtype=np.uint64)]
    rows = len(rp) - 1
    if pieces < 1:
        raise ValueError("pieces must be >= 1")
    nnz = rp[-1] if rows >= 0 else 0
    per_row = max(nnz, rows)
    total = nnz * rows + rows * per_row
    bounds = []
    for i in range(pieces + 1):
        target = total * i // pieces
        lo, hi = 0, rows
        while lo < hi:
            mid = (lo + hi) // 2
            if rp[mid] * rows + mid * per_row >= target:
                hi = mid
            else:
                lo = mid + 1
        bounds.append(lo)
    bounds[0], bounds[-1] = 0, rows
    return np.maximum.accumulate(np.array(bounds, dtype=np.uint64))


def exchange_slots(slots, world: int, rank: int, chunks: int, group=None) -> None:
    """All-gather the gathered-Y slots of an external-context matrix over a
    torch.distributed group: rank r's slots c*world + r (c < chunks) go to
    every rank, in place, as ncclAllGather would put them.

    `slots` has ``slot_read(first, n) -> (y, nz)`` and ``slot_write(first, y,
    nz)`` (``MultiCsr`` or a host stand-in), host numpy arrays shaped (n,
    piece_rows, k) and (n, piece_rows)."""
    import torch
    import torch.distributed as dist

    mine_y, mine_nz = [], []
    for c in range(chunks):
        y, nz = slots.slot_read(c * world + rank, 1)
        mine_y.append(y[0])
        mine_nz.append(nz[0])
    ty = torch.from_numpy(np.ascontiguousarray(np.stack(mine_y)))
    tn = torch.from_numpy(np.ascontiguousarray(np.stack(mine_nz)))
    # gloo gathers raw bytes fine; view floats as same-width integers so no
    # backend ever touches the values (NaN payloads, -0.0 stay as they are)
    iview = {8: torch.int64, 4: torch.int32, 2: torch.int16, 1: torch.uint8}[ty.element_size()]
    ty_i = ty.view(iview)
    all_y = [torch.empty_like(ty_i) for _ in range(world)]
    all_n = [torch.empty_like(tn) for _ in range(world)]
    dist.all_gather(all_y, ty_i, group=group)
    dist.all_gather(all_n, tn, group=group)
    for r in range(world):
        if r == rank:
            continue
        yr = all_y[r].view(ty.dtype).numpy()
        nr = all_n[r].numpy()
        for c in range(chunks):
            slots.slot_write(c * world + r, yr[c:c + 1], nr[c:c + 1])


class HostSlots:
    """Host stand-in of a matrix's gathered-Y slots (P slots of piece_rows x k),
    with MultiCsr's slot_read / slot_write interface (CPU tests)."""

    def __init__(self, pieces: int, piece_rows: int, k: int, dtype=np.float64):
        self.y = np.zeros((pieces, piece_rows, k), dtype=dtype)
        self.nz = np.zeros((pieces, piece_rows), dtype=np.int32)

    def slot_read(self, first: int, n: int):
        return self.y[first:first + n].copy(), self.nz[first:first + n].copy()

    def slot_write(self, first: int, y, nz) -> None:
        self.y[first:first + len(y)] = y
        self.nz[first:first + len(nz)] = nz

    def assembled(self, bounds) -> tuple:
        """Y (rows x k) and row counts in global row order (bsm_mcsr_copy_y)."""
        b = np.asarray(bounds, dtype=np.int64)
        ys = [self.y[i, :b[i + 1] - b[i]] for i in range(len(b) - 1)]
        ns = [self.nz[i, :b[i + 1] - b[i]] for i in range(len(b) - 1)]
        return np.concatenate(ys), np.concatenate(ns)
