"""The N > 1 row split on CPU (gloo, world_size 2 and 3).

* The piece bounds: the Python restatement (distributed.partition_rows) equals
  the library's own (bsm_partition_rows, a host-only C-ABI call, no device),
  and the bounds keep every piece under 2*rows/P + 1 rows on skewed matrices
  (a pure nnz split let one piece take nearly every row).
* The slot exchange of an external context (distributed.exchange_slots over
  gloo), driven with host stand-ins of the gathered-Y slots that each rank
  fills with the oracle's Y for its own pieces (the GPU kernel's per-row
  bit-exactness is covered by the -m gpu tests; tests/test_gpu_distributed.py
  runs this same exchange on the library's device slots). After the exchange
  every rank must hold the single-process Y bit for bit, padding rows zero.
Rows are independent in the reference (src/sparse.rs:431-444), so the split
cannot change a bit.
"""

import os
import socket

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp

from basic_sparse_matrix_amd import _lib
from basic_sparse_matrix_amd.distributed import HostSlots, exchange_slots, partition_rows


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _dense_y(orc, n_cols, rp, ci, v, x_cols, r0, r1):
    """Oracle Y for rows [r0, r1) as a dense (r1-r0) x k array and its counts."""
    k = len(x_cols)
    lrp = (rp[r0:r1 + 1] - rp[r0]).astype(np.uint64)
    lo, hi = int(rp[r0]), int(rp[r1])
    orp, oci, ov = orc.mul_dense(r1 - r0, n_cols, lrp, ci[lo:hi], v[lo:hi], x_cols)
    y = np.zeros((r1 - r0, k))
    rows_of = np.repeat(np.arange(r1 - r0), np.diff(orp.astype(np.int64)))
    y[rows_of, oci.astype(np.int64)] = ov
    return y, np.diff(orp.astype(np.int64)).astype(np.int32)


def _row_ptrs():
    rng = np.random.default_rng(7)
    cases = []
    for lens in (
        rng.integers(0, 40, 997),                                   # uniform lengths: unequal pieces
        np.full(1000, 20),                                          # equal lengths (C4's shape)
        np.concatenate([np.zeros(9000, np.int64), np.full(1000, 100)]),  # long empty run
        np.concatenate([[10**6], np.ones(5000, np.int64)]),         # one huge row first
        np.concatenate([np.ones(5000, np.int64), [10**6]]),         # one huge row last
        (rng.pareto(1.2, 3000) * 3).astype(np.int64),               # power law
        np.zeros(50, np.int64),                                     # empty matrix
        np.zeros(0, np.int64),                                      # no rows
        np.array([3, 0, 0, 5]),
    ):
        cases.append(np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64))
    return cases


@pytest.mark.parametrize("case", range(9))
def test_partition_mirror_equals_library_and_caps_rows(case):
    rp = _row_ptrs()[case]
    rows = rp.size - 1
    lib_ok = True
    try:
        _lib.load()
    except _lib.DeviceUnavailable:
        lib_ok = False  # library not built: the mirror's properties are still checked
    from basic_sparse_matrix_amd.multi import partition_rows as lib_partition

    for P in (1, 2, 3, 4, 8, 12, 32):
        b = partition_rows(rp, P)
        assert b[0] == 0 and b[-1] == rows and np.all(np.diff(b.astype(np.int64)) >= 0)
        if lib_ok:
            assert np.array_equal(lib_partition(rp, P), b), (case, P)
        pad = int(np.max(np.diff(b.astype(np.int64)))) if rows else 0
        assert pad <= 2 * rows / P + 1, (case, P, pad)
        lens = np.diff(rp.astype(np.int64))
        if rows and np.all(lens == lens[0]) and lens[0] > 0:
            # equal row lengths: the cost split is the nnz split (bound i = first
            # row starting at or past i*nnz/P)
            nnz = int(rp[-1])
            want = np.searchsorted(rp[:-1].astype(np.int64), [nnz * i // P for i in range(P + 1)], side="left")
            want[0], want[-1] = 0, rows
            assert np.array_equal(b.astype(np.int64), np.maximum.accumulate(want)), (case, P)


def _worker(rank, world, port, chunks, rows, kind, result_q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from oracle import pyoracle as orc

    n_cols, k = 700, 5
    rp, ci, v = orc.gen_csr(1000, rows, n_cols, kind, 0 if kind else 12, 30 if kind else 12)
    x_cols = orc.gen_x_cols(1001, n_cols, k)
    P = chunks * world
    b = partition_rows(rp, P).astype(np.int64)
    pad = int(np.max(np.diff(b))) if rows else 0
    slots = HostSlots(P, pad, k)
    # this rank's rounds (what bsm_mcsr_step writes on an external context);
    # the other slots hold garbage the exchange must overwrite
    slots.y[:] = np.nan
    slots.nz[:] = -7
    for c in range(chunks):
        p = c * world + rank
        y, nz = _dense_y(orc, n_cols, rp, ci, v, x_cols, int(b[p]), int(b[p + 1]))
        slots.y[p] = 0.0
        slots.nz[p] = 0
        slots.y[p, :len(y)] = y
        slots.nz[p, :len(nz)] = nz
    exchange_slots(slots, world, rank, chunks)
    y_all, nz_all = slots.assembled(b)
    ref_y, ref_nz = _dense_y(orc, n_cols, rp, ci, v, x_cols, 0, rows)
    ok = bool(np.array_equal(y_all.view(np.uint64), ref_y.view(np.uint64)) and np.array_equal(nz_all, ref_nz))
    # slot rows past a piece's end: zero values, zero counts (what compaction skips)
    for p in range(P):
        n = int(b[p + 1] - b[p])
        ok &= bool(np.all(slots.y[p, n:] == 0) and np.all(slots.nz[p, n:] == 0))
    oks = [None] * world
    dist.all_gather_object(oks, ok)
    if rank == 0:
        result_q.put(all(oks))
    dist.barrier()
    dist.destroy_process_group()


def test_partition_rows_rejects_empty_row_ptr():
    """row_ptr holds rows + 1 entries; an empty array is refused in Python
    (the C entry point trusts rows)."""
    from basic_sparse_matrix_amd.multi import partition_rows as lib_partition

    with pytest.raises(ValueError):
        lib_partition(np.zeros(0, dtype=np.uint64), 4)


@pytest.mark.parametrize("world,chunks,rows,kind", [
    (2, 1, 997, 1), (2, 3, 997, 1), (3, 1, 601, 1), (3, 4, 1000, 1),
    (3, 2, 600, 0),   # equal pieces
    (2, 4, 5, 1),     # more pieces than rows: empty pieces
])
def test_exchange_slots_gloo_matches_single(world, chunks, rows, kind):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, chunks, rows, kind, q)) for r in range(world)]
    for p in procs:
        p.start()
    for p in procs:
        p.join(120)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    assert q.get(timeout=5) is True
