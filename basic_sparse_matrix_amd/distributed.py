"""Row-block multi-GPU SpMM (BASELINE.json north_star).

One process per GPU (torch.distributed, backend "nccl" = RCCL over xGMI).
The CSR is split into contiguous row blocks of (nearly) equal nnz; the dense
RHS X is replicated on every rank; each rank computes its block of Y = A X
with the local HIP kernels, and the full dense Y is assembled on every rank
with ONE all-gather (equal-count blocks, padded). Per-row results do not
depend on the partition (each row is reduced by one wavefront in entry
order), so the assembled Y is bit-identical to the single-GPU one.

Only the partitioning / padding / assembly logic lives here; it is used by
bench.py on GPUs and by tests/test_distributed_cpu.py with the gloo backend.
"""

from __future__ import annotations

import numpy as np


def partition_rows_by_nnz(row_ptr, world: int) -> np.ndarray:
    """Contiguous row bounds (world+1 entries) splitting nnz as evenly as a
    row boundary allows: bound g is the first row whose start >= g*nnz/world
    (binary search on row_ptr). Empty matrices split rows evenly."""
    rp = np.asarray(row_ptr, dtype=np.int64)
    rows = len(rp) - 1
    nnz = int(rp[-1]) if rows >= 0 else 0
    if world < 1:
        raise ValueError("world must be >= 1")
    if nnz == 0:
        return np.array([(rows * g) // world for g in range(world + 1)], dtype=np.int64)
    targets = [(nnz * g) // world for g in range(world + 1)]
    bounds = np.searchsorted(rp[:-1], targets, side="left").astype(np.int64)
    bounds[0], bounds[-1] = 0, rows
    return np.maximum.accumulate(bounds)


def partition_rows_even(rows: int, world: int) -> np.ndarray:
    """Equal row counts (equal nnz when every row has the same length, as in
    the C4 bench matrix); the last block is the short one."""
    per = (rows + world - 1) // world
    return np.array([min(rows, g * per) for g in range(world + 1)], dtype=np.int64)


def padded_block_rows(bounds) -> int:
    b = np.asarray(bounds)
    return int(np.max(np.diff(b))) if len(b) > 1 else 0


def all_gather_blocks(y_local_padded, group=None):
    """All-gather equal-size (pad_rows x k) blocks -> (world*pad_rows x k)."""
    import torch
    import torch.distributed as dist

    world = dist.get_world_size(group)
    out = torch.empty((world * y_local_padded.shape[0],) + tuple(y_local_padded.shape[1:]),
                      dtype=y_local_padded.dtype, device=y_local_padded.device)
    dist.all_gather_into_tensor(out, y_local_padded.contiguous(), group=group)
    return out


def unpad_blocks(y_gathered, bounds, pad_rows: int):
    """Drop the padding rows of each gathered block -> (rows x k)."""
    import torch

    b = np.asarray(bounds)
    world = len(b) - 1
    if world == 1 or np.all(np.diff(b)[:-1] == pad_rows):
        return y_gathered[: int(b[-1])]  # only the last block can be short
    parts = [y_gathered[g * pad_rows: g * pad_rows + int(b[g + 1] - b[g])] for g in range(world)]
    return torch.cat(parts, dim=0)


def partition_rows_cyclic(rows: int, world: int, chunks: int):
    """Block-cyclic row partition for an all-gather overlapped with compute.

    The rows are cut into `chunks` rounds of world*cr consecutive rows
    (cr = ceil(rows / (chunks*world))); in round c rank g owns rows
    [c*world*cr + g*cr, ... + cr), clipped to `rows`. Round c of every rank
    is finished by the same SpMM launch, and the equal-count all-gather of
    round c lands contiguously, already in global row order, at rows
    [c*world*cr, (c+1)*world*cr) of the gathered buffer: no reordering copy,
    and only the last round holds padding (rows >= `rows`, never read).

    Returns (cr, [[(row0, nrows) for c in range(chunks)] for g in range(world)]);
    nrows may be 0 for trailing pieces."""
    if world < 1 or chunks < 1:
        raise ValueError("world and chunks must be >= 1")
    cr = -(-rows // (chunks * world)) if rows else 0
    pieces = []
    for g in range(world):
        mine = []
        for c in range(chunks):
            r0 = c * world * cr + g * cr
            mine.append((min(r0, rows), max(0, min(rows, r0 + cr) - r0)))
        pieces.append(mine)
    return cr, pieces
