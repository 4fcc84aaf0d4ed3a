"""Multi-rank path on CPU (gloo, world_size 2 and 3): row-block partition,
padded all-gather and assembly give exactly the single-process result.

Each rank computes its block of Y = A X with the CPU oracle (a stand-in for
the GPU kernel, whose per-row bit-exactness is covered by the GPU tests); the
assembly code under test is the same module bench.py uses on RCCL.
"""

import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

from basic_sparse_matrix_amd.distributed import (all_gather_blocks, padded_block_rows, partition_rows_by_nnz,
                                                 partition_rows_even, unpad_blocks)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dense_y(orc, rows, n_cols, rp, ci, v, x_cols, r0, r1):
    """Oracle Y for rows [r0, r1) as a dense (r1-r0) x k array."""
    k = len(x_cols)
    lrp = (rp[r0:r1 + 1] - rp[r0]).astype(np.uint64)
    lo, hi = int(rp[r0]), int(rp[r1])
    orp, oci, ov = orc.mul_dense(r1 - r0, n_cols, lrp, ci[lo:hi], v[lo:hi], x_cols)
    y = np.zeros((r1 - r0, k))
    rows_of = np.repeat(np.arange(r1 - r0), np.diff(orp.astype(np.int64)))
    y[rows_of, oci.astype(np.int64)] = ov
    return y


def _worker(rank, world, port, even, result_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import pyoracle as orc

    rows, n_cols, k = 997, 800, 5
    rp, ci, v = orc.gen_csr(1000, rows, n_cols, orc.ROWLEN_UNIFORM, 0, 30)
    x_cols = orc.gen_x_cols(1001, n_cols, k)
    bounds = partition_rows_even(rows, world) if even else partition_rows_by_nnz(rp, world)
    pad = padded_block_rows(bounds)
    r0, r1 = int(bounds[rank]), int(bounds[rank + 1])
    y_local = torch.zeros((pad, k), dtype=torch.float64)
    y_local[: r1 - r0] = torch.from_numpy(_dense_y(orc, rows, n_cols, rp, ci, v, x_cols, r0, r1))
    y_full = unpad_blocks(all_gather_blocks(y_local), bounds, pad)
    if rank == 0:
        ref = _dense_y(orc, rows, n_cols, rp, ci, v, x_cols, 0, rows)
        result_q.put(bool(np.array_equal(y_full.numpy().view(np.uint64), ref.view(np.uint64))))
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,even", [(2, True), (2, False), (3, False)])
def test_row_block_allgather_matches_single(world, even):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, even, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True


def test_partition_by_nnz_balanced():
    lens = np.array([5, 0, 0, 100, 1, 1, 1, 50, 3, 0, 40], dtype=np.int64)
    rp = np.concatenate([[0], np.cumsum(lens)])
    for world in (1, 2, 3, 4, 8):
        b = partition_rows_by_nnz(rp, world)
        assert b[0] == 0 and b[-1] == len(lens) and np.all(np.diff(b) >= 0)
    b = partition_rows_even(10_000_000, 8)
    assert list(np.diff(b)) == [1_250_000] * 8
    b = partition_rows_even(10, 4)
    assert list(b) == [0, 3, 6, 9, 10]
    assert padded_block_rows(b) == 3
