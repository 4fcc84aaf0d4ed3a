"""One rank of the library's multi-GPU Csr::mul_dense at world > 1 on ONE GPU
(launched as a fresh child process by tests/test_gpu_distributed.py; not a
test module itself).

Each rank makes an external context (bsm_multi_create_external: rank r of
world on cuda:0, no RCCL communicator, since RCCL allows one rank per
device) and the partitioned matrix (bsm_mcsr_upload of the oracle's host
arrays, or bsm_mcsr_generate on the device), prepares the schedule asked
for, runs bsm_mcsr_step (this rank's rounds into its slots c*world + r of the
gathered Y), exchanges the slots with the other ranks over gloo
(distributed.exchange_slots: what the in-place ncclAllGather of the RCCL path
leaves), and compacts with bsm_mcsr_compact. So the library's own rank != 0
slot placement, slot padding, row_ptr squeeze and compaction run with
several ranks. Every rank's output Csr must be the same; rank 0 checks it
bit for bit against the single-GPU bsm_csr_mul_dense and the CPU oracle
(Csr::mul_dense, src/sparse.rs:426-446). The verdict goes to argv[1] as
JSON.

argv: out_json mode(upload|generate) rows n_cols kind a b k chunks schedule(auto|tiled|panel) dtype(f64|f32|i32)
env DIST_OUTPUT_RANK=r: only rank r compacts and returns the output Csr
(bsm_mcsr_set_output_rank); the other ranks must refuse bsm_mcsr_output.
"""

import hashlib
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402


def bits(a):
    a = np.asarray(a)
    return a.view(np.uint64 if a.dtype.itemsize == 8 else np.uint32) if a.dtype.kind == "f" else a


def same_csr(got, want):
    rp, ci, v = got
    erp, eci, ev = want
    return bool(np.array_equal(np.asarray(rp, np.uint64), np.asarray(erp, np.uint64))
                and np.array_equal(np.asarray(ci, np.uint64), np.asarray(eci, np.uint64))
                and np.array_equal(bits(v), bits(np.asarray(ev, dtype=np.asarray(v).dtype))))


def main():
    out_json, mode = sys.argv[1], sys.argv[2]
    rows, n_cols, kind, a, b, k, chunks = (int(x) for x in sys.argv[3:10])
    schedule, dts = sys.argv[10], sys.argv[11]
    dtype = {"f64": np.float64, "f32": np.float32, "i32": np.int32}[dts]
    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)  # every rank shares the one GPU of the box
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", rank=rank, world_size=world)

    from basic_sparse_matrix_amd import Csr, Dense, _lib
    from basic_sparse_matrix_amd.device import DeviceCsrBlock, gen_dense
    from basic_sparse_matrix_amd.distributed import exchange_slots, partition_rows
    from basic_sparse_matrix_amd.multi import MultiCsr, MultiGpu
    from oracle import pyoracle as orc

    ctx = MultiGpu.external(world, rank, 0)
    assert ctx.is_external and (ctx.world, ctx.n_local, ctx.first_rank) == (world, 1, rank)
    vk = 1 if np.dtype(dtype).kind == "i" else 0
    res = {"rank": rank}
    if mode == "upload":
        rp, ci, v = orc.gen_csr(1000, rows, n_cols, kind, a, b, vk, dtype=np.float64)
        v = v.astype(dtype)
        x_cols = [c.astype(dtype) for c in orc.gen_x_cols(1001, n_cols, k, value_kind=vk)]
        m = MultiCsr.upload(ctx, rows, n_cols, rp, ci, v, chunks=chunks)
        x = torch.from_numpy(np.ascontiguousarray(np.stack(x_cols, axis=1) if k else
                                                  np.zeros((n_cols, 0), dtype))).to(dev)
        res["bounds_equal_mirror"] = bool(np.array_equal(m.bounds(), partition_rows(rp, chunks * world)))
    else:
        assert dtype == np.float64, "generate mode: f64 (the bench's matrices)"
        m = MultiCsr.generate(ctx, 1000, rows, n_cols, kind, a, b, 0, dtype, chunks=chunks)
        x = gen_dense(1001, 0, n_cols, k, device=dev)
    assert m.pieces == chunks * world
    res["pieces"], res["piece_rows"] = m.pieces, m.piece_rows
    bd = m.bounds().astype(np.int64)
    res["squeeze"] = bool(np.any(np.diff(bd)[:-1] != m.piece_rows))
    res["empty_pieces"] = int(np.sum(np.diff(bd) == 0))
    out_rank = int(os.environ.get("DIST_OUTPUT_RANK", "-1"))
    if out_rank >= 0:
        m.set_output_rank(out_rank)
    m.prepare(k, schedule)
    res["plan"] = m.plan_info()
    root = out_rank if out_rank >= 0 else 0
    torch.cuda.synchronize()
    outs = []
    holds_output = out_rank < 0 or rank == out_rank
    for it in range(2):  # a second step over the slots of the first exchange
        m.step([x.data_ptr()])
        m.sync()
        exchange_slots(m, world, rank, chunks)
        m.compact()
        m.sync()
        if holds_output:
            outs.append(m.output().download())
    if holds_output:
        got = outs[-1]
        res["steps_equal"] = same_csr(outs[0], got)
        h = hashlib.sha256()
        for arr in got:
            h.update(np.ascontiguousarray(arr).tobytes())
        digest = h.hexdigest()
    else:  # no output here: bsm_mcsr_output must refuse
        try:
            m.output()
            res["steps_equal"] = False
        except _lib.BsmError:
            res["steps_equal"] = True
        digest = None
    digests = [None] * world
    dist.all_gather_object(digests, digest)
    res["ranks_agree"] = len({d for d in digests if d is not None}) == 1 and (out_rank < 0 or digests.count(None) == world - 1)
    if rank == root:
        if mode == "upload":
            want = orc.mul_dense(rows, n_cols, rp, ci, v, x_cols)
            res["oracle_equal"] = same_csr(got, want)
            single = Csr.from_csr_arrays((rows, n_cols), rp, ci, v).mul_dense(
                Dense.from_columns(x_cols) if k else Dense(0, n_cols, []))
            res["single_equal"] = same_csr((single.row_index, single.col_index, single.v), want)
        else:
            # the assembled Y (slot order -> row order) against one block on
            # the single-GPU kernel, and sampled rows against the oracle
            tdt = torch.float64
            y = torch.empty((rows, k), dtype=tdt, device=dev)
            nz = torch.empty(rows, dtype=torch.int32, device=dev)
            m.copy_y(0, y.data_ptr(), nz.data_ptr())
            blk = DeviceCsrBlock.generate(1000, 0, rows, n_cols, kind, a, b, 0, dtype, device=dev)
            y_ref = torch.empty((rows, k), dtype=tdt, device=dev)
            nz_ref = torch.empty(rows, dtype=torch.int32, device=dev)
            blk.spmm(x, y_ref, nz_ref)
            torch.cuda.synchronize()
            res["single_equal"] = bool(torch.equal(y.view(torch.int64), y_ref.view(torch.int64))
                                       and torch.equal(nz, nz_ref))
            rp_o, ci_o, v_o = got
            grp = orc.gen_row_ptr(1000, rows, n_cols, kind, a, b)
            xc = orc.gen_x_cols(1001, n_cols, k)
            ok = int(rp_o[-1]) == int(nz_ref.sum().item())
            for r in np.linspace(0, rows - 1, 60).astype(np.int64):
                gci, gv = orc.gen_entries(1000, grp, n_cols, r0=int(r), r1=int(r) + 1)
                a0, a1 = int(grp[r]), int(grp[r + 1])
                srp = np.array([0, a1 - a0], np.uint64)
                erp, eci, ev = orc.mul_dense(1, n_cols, srp, gci[a0:a1], gv[a0:a1], xc)
                o0, o1 = int(rp_o[r]), int(rp_o[r + 1])
                ok &= bool(np.array_equal(ci_o[o0:o1], eci) and np.array_equal(bits(v_o[o0:o1]), bits(ev)))
            res["oracle_equal"] = ok
    dist.barrier()
    del m
    ctx.close()
    dist.destroy_process_group()
    with open(out_json, "w") as f:
        json.dump(res, f)


if __name__ == "__main__":
    main()
