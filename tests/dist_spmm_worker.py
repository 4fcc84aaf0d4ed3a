"""One rank of the multi-rank SpMM path that bench.py --gpus N runs
(launched as a fresh child process by tests/test_gpu_distributed.py; not a
test module itself).

Each rank generates its block-cyclic row pieces on the device
(partition_rows_cyclic + DeviceCsrBlock.generate), runs the HIP SpMM on each
piece (optionally with the column-panel plan), and all-gathers Y and the
per-row nonzero counts round by round with async collectives, exactly as
bench.py's step does. Rank 0 then recomputes the whole product on its own
GPU in one piece and compares bit for bit, compacts the assembled Y into the
output Csr, and checks a sampled row range against the CPU oracle
(Csr::mul_dense, src/sparse.rs:426-446). The verdict is written as JSON to
argv[1].

argv: out_json rows n_cols nnz_per_row k chunks panel_cols(0 = none, -1 = the
tiled row-block x column-panel copy, forced, per piece)
"""

import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def main():
    out_json = sys.argv[1]
    rows, n_cols, nnz_r, k, chunks, panel = (int(a) for a in sys.argv[2:8])
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)  # every rank shares the one GPU of the box
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    from basic_sparse_matrix_amd import _lib
    from basic_sparse_matrix_amd.device import Compactor, DeviceCsrBlock, gen_dense
    from basic_sparse_matrix_amd.distributed import partition_rows_cyclic

    cr, pieces = partition_rows_cyclic(rows, world, chunks)
    blks = [DeviceCsrBlock.generate(1000, r0, n, n_cols, _lib.ROWLEN_UNIFORM, 0, 2 * nnz_r, _lib.VAL_UNIFORM,
                                    np.float64, device=dev) for r0, n in pieces[rank]]
    if panel == -1:
        widths = [-1 if b.nnz and b.plan_tiled(k, force=True) is not None else 0 for b in blks]
    else:
        widths = [b.plan(k, panel) if panel else 0 for b in blks]
    x = gen_dense(1001, 0, n_cols, k, device=dev)
    y_local = torch.full((chunks, cr, k), float("nan"), dtype=torch.float64, device=dev)
    nnz_local = torch.full((chunks, cr), -1, dtype=torch.int32, device=dev)
    y_full = torch.empty((chunks * world * cr, k), dtype=torch.float64, device=dev)
    nnz_full = torch.empty(chunks * world * cr, dtype=torch.int32, device=dev)
    works = []
    rr = world * cr
    for c, b in enumerate(blks):
        if b.rows:
            b.spmm(x, y_local[c, :b.rows], nnz_local[c, :b.rows])
        torch.cuda.synchronize()  # gloo reads the tensors from the host side
        works.append(dist.all_gather_into_tensor(y_full[c * rr:(c + 1) * rr], y_local[c], async_op=True))
        works.append(dist.all_gather_into_tensor(nnz_full[c * rr:(c + 1) * rr], nnz_local[c], async_op=True))
    for w in works:
        w.wait()
    torch.cuda.synchronize()
    res = {"rank": rank, "widths": widths}
    if rank == 0:
        full = DeviceCsrBlock.generate(1000, 0, rows, n_cols, _lib.ROWLEN_UNIFORM, 0, 2 * nnz_r, _lib.VAL_UNIFORM,
                                       np.float64, device=dev)
        y_ref = torch.empty((rows, k), dtype=torch.float64, device=dev)
        nnz_ref = torch.empty(rows, dtype=torch.int32, device=dev)
        full.spmm(x, y_ref, nnz_ref)
        torch.cuda.synchronize()
        res["y_equal"] = bool(torch.equal(y_ref.view(torch.int64), y_full[:rows].view(torch.int64)))
        res["nnz_equal"] = bool(torch.equal(nnz_ref, nnz_full[:rows]))
        comp = Compactor(rows, k, np.float64, device=dev)
        comp(y_full[:rows], nnz_full[:rows])
        torch.cuda.synchronize()
        # oracle on a sampled row range of the assembled, compacted product
        from oracle import pyoracle as orc

        s0, sn = rows // 3, min(300, rows - rows // 3)
        frp = orc.gen_row_ptr(1000, rows, n_cols, orc.ROWLEN_UNIFORM, 0, 2 * nnz_r)
        ci, v = orc.gen_entries(1000, frp, n_cols, r0=s0, r1=s0 + sn)
        lo, hi = int(frp[s0]), int(frp[s0 + sn])
        lrp = (frp[s0:s0 + sn + 1] - frp[s0]).astype(np.uint64)
        x_cols = orc.gen_x_cols(1001, n_cols, k)
        erp, eci, ev = orc.mul_dense(sn, n_cols, lrp, ci[lo:hi], v[lo:hi], x_cols)
        crp = comp.row_ptr.cpu().numpy()
        a, e = int(crp[s0]), int(crp[s0 + sn])
        res["oracle_rows"] = [s0, s0 + sn]
        res["oracle_equal"] = bool(
            np.array_equal((crp[s0:s0 + sn + 1] - crp[s0]).astype(np.uint64), erp)
            and np.array_equal(comp.col[a:e].cpu().numpy().astype(np.uint64), eci)
            and np.array_equal(comp.vals[a:e].cpu().numpy().view(np.uint64), ev.view(np.uint64)))
        res["out_nnz"] = comp.nnz()
    dist.barrier()
    dist.destroy_process_group()
    with open(out_json, "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()
