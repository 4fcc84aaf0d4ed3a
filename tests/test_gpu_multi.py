"""GPU parity of the multi-GPU Csr::mul_dense behind the C-ABI
(include/bsm.h "multi-GPU", csrc/multi.hip; north_star: row blocks on every
GPU + RCCL all-gather; reference src/sparse.rs:426-446).

One GPU is visible here, so the communicator has one rank; the RCCL calls
(ncclCommInitAll / ncclCommInitRank, in-place ncclAllGather per round,
ncclBroadcast) still run, through the same code as at N = 8. Every result is
compared BIT-EXACT with the oracle (oracle/, the C restatement of
sparse.rs:426-446) and with the single-GPU bsm_csr_mul_dense: the pieces,
their padding and the round structure must not change a bit. The last test
launches bench.py under torch.distributed.run with the nccl backend, so
torch's RCCL collectives (the id broadcast, barriers, the max all-reduce) and
the library's all-gathers both execute on the GPU.
"""

import json
import os
import socket
import subprocess
import sys

import numpy as np
import pytest
import torch

import basic_sparse_matrix_amd as bsm
from basic_sparse_matrix_amd import Csr, Dense, Panic, _lib
from basic_sparse_matrix_amd.device import DeviceCsrBlock, gen_dense
from basic_sparse_matrix_amd.multi import MultiCsr, MultiGpu, unique_id

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bits(a):
    a = np.asarray(a)
    if a.dtype.kind == "f":
        return a.view(np.uint64 if a.dtype.itemsize == 8 else np.uint32)
    return a


def assert_same_csr(got, want):
    rp, ci, v = got
    erp, eci, ev = want
    assert np.array_equal(np.asarray(rp, np.uint64), np.asarray(erp, np.uint64)), "row_ptr differs"
    assert np.array_equal(np.asarray(ci, np.uint64), np.asarray(eci, np.uint64)), "col_idx differs"
    assert np.array_equal(bits(v), bits(np.asarray(ev, dtype=np.asarray(v).dtype))), "values differ"


@pytest.fixture(autouse=True)
def _rccl_at_one_rank(monkeypatch):
    """At one rank the step skips the all-gathers (nothing to move); these
    tests run them anyway, so the RCCL calls execute on the GPU."""
    monkeypatch.setenv("BSM_MULTI_SOLO_RCCL", "1")


@pytest.fixture(scope="module")
def ctx():
    c = MultiGpu(1)
    yield c
    c.close()


def make(orc, rows, cols, kind, a, b, dtype, seed=1000, value_kind=0):
    """Seeded random CSR; row lengths uniform in [a, b] (a = 0: empty rows too),
    so nnz-balanced pieces have unequal row counts (slot padding + squeeze)."""
    rp, ci, v = orc.gen_csr(seed, rows, cols, kind, a, b, value_kind, dtype=np.float64)
    return rp, ci, v.astype(dtype)


CASES = [
    # rows, cols, kind, a, b, k, chunks, dtype
    (3000, 2000, 1, 0, 40, 32, 1, np.float64),
    (3000, 2000, 1, 0, 40, 32, 4, np.float64),   # unequal pieces: slot padding + row_ptr squeeze
    (1000, 5000, 1, 0, 7, 1, 3, np.float64),
    (777, 513, 1, 0, 20, 5, 2, np.float32),
    (500, 400, 1, 1, 9, 3, 5, np.int32),
    (64, 64, 1, 0, 3, 0, 2, np.float64),          # k = 0: every output row empty
    (10, 30, 1, 0, 12, 2, 16, np.float64),        # more pieces than rows: empty pieces
    (2000, 3000, 0, 20, 20, 32, 4, np.float64),   # equal pieces: no squeeze
]


@pytest.mark.parametrize("rows,cols,kind,a,b,k,chunks,dtype", CASES)
def test_multi_g1_matches_oracle_and_single_gpu(ctx, orc, rows, cols, kind, a, b, k, chunks, dtype):
    vk = 1 if np.dtype(dtype).kind == "i" else 0
    rp, ci, v = make(orc, rows, cols, kind, a, b, dtype, value_kind=vk)
    x_cols = [c.astype(dtype) for c in orc.gen_x_cols(1001, cols, k, value_kind=vk)]
    m = MultiCsr.upload(ctx, rows, cols, rp, ci, v, chunks=chunks)
    assert m.pieces == chunks and m.nnz == int(rp[-1])
    bd = m.bounds()
    assert bd[0] == 0 and bd[-1] == rows and np.all(np.diff(bd.astype(np.int64)) >= 0)
    got = m.mul_dense_cols(x_cols, cols).download()
    want = orc.mul_dense(rows, cols, rp, ci, v, x_cols)
    assert_same_csr(got, want)
    single = Csr.from_csr_arrays((rows, cols), rp, ci, v).mul_dense(Dense.from_columns(x_cols) if k else
                                                                     Dense(0, cols, []))
    assert_same_csr((single.row_index, single.col_index, single.v), want)
    # a second call on the prepared handle gives the same bits
    assert_same_csr(m.mul_dense_cols(x_cols, cols).download(), want)


def test_multi_rank_mode_world1(orc):
    """One process per GPU: ncclCommInitRank from a shipped id (world 1)."""
    c = MultiGpu.for_rank(unique_id(), 1, 0, 0)
    assert (c.world, c.n_local, c.first_rank) == (1, 1, 0)
    rp, ci, v = orc.gen_csr(1000, 2000, 3000, 1, 0, 30)
    x_cols = orc.gen_x_cols(1001, 3000, 32)
    m = MultiCsr.upload(c, 2000, 3000, rp, ci, v, chunks=3)
    assert_same_csr(m.mul_dense_cols(x_cols, 3000).download(), orc.mul_dense(2000, 3000, rp, ci, v, x_cols))
    del m
    c.close()


@pytest.mark.parametrize("schedule,chunks", [("tiled", 3), ("panel", 2), ("auto", 1)])
def test_multi_generate_step_matches_device_block(ctx, orc, schedule, chunks):
    """The bench's device-level path: pieces generated on the device, X
    broadcast, step/sync, the assembled Y and the compacted Csr checked
    against one block computed by the one-pass kernel, and 40 rows against the
    oracle."""
    rows, n_cols, nnz_r, k = 20000, 30000, 50, 32
    dev = torch.device("cuda", 0)
    m = MultiCsr.generate(ctx, 1000, rows, n_cols, _lib.ROWLEN_CONST, nnz_r, nnz_r, 0, np.float64, chunks=chunks)
    assert m.nnz == rows * nnz_r
    plan = m.prepare(k, schedule)
    info = m.plan_info()
    assert info["local_pieces"] == chunks
    if schedule == "tiled":
        assert info["tiled_pieces"] == chunks and info["copy_bytes"] > 0 and plan["tiled_write"] >= 0
    if schedule == "panel":
        assert info["tiled_pieces"] == 0
    x = torch.empty((n_cols, k), dtype=torch.float64, device=dev)
    x.copy_(gen_dense(1001, 0, n_cols, k, device=dev))
    torch.cuda.synchronize()
    ctx.broadcast([x.data_ptr()], x.numel() * 8, 0)
    for _ in range(3):
        m.step([x.data_ptr()])
    m.sync()
    ts = m.step_times(0)
    assert len(ts) == 3 and all(t["spmm"] > 0 and t["total"] >= t["spmm"] for t in ts)
    y = torch.empty((rows, k), dtype=torch.float64, device=dev)
    nz = torch.empty(rows, dtype=torch.int32, device=dev)
    m.copy_y(0, y.data_ptr(), nz.data_ptr())
    blk = DeviceCsrBlock.generate(1000, 0, rows, n_cols, _lib.ROWLEN_CONST, nnz_r, nnz_r, 0, np.float64, device=dev)
    y_ref = torch.empty((rows, k), dtype=torch.float64, device=dev)
    nz_ref = torch.empty(rows, dtype=torch.int32, device=dev)
    blk.spmm(x, y_ref, nz_ref)
    torch.cuda.synchronize()
    assert torch.equal(y.view(torch.int64), y_ref.view(torch.int64))
    assert torch.equal(nz, nz_ref)
    out = m.output()
    rp, ci, v = out.download()
    assert int(rp[-1]) == int(nz_ref.sum().item())
    # oracle on 40 sampled rows
    sel = np.linspace(0, rows - 1, 40).astype(np.int64)
    grp = orc.gen_row_ptr(1000, rows, n_cols, _lib.ROWLEN_CONST, nnz_r, nnz_r)
    gci, gv = orc.gen_entries(1000, grp, n_cols)
    x_cols = orc.gen_x_cols(1001, n_cols, k)
    for r in sel:
        a0, a1 = int(grp[r]), int(grp[r + 1])
        srp = np.array([0, a1 - a0], np.uint64)
        erp, eci, ev = orc.mul_dense(1, n_cols, srp, gci[a0:a1], gv[a0:a1], x_cols)
        o0, o1 = int(rp[r]), int(rp[r + 1])
        assert np.array_equal(ci[o0:o1], eci) and np.array_equal(bits(v[o0:o1]), bits(ev)), f"row {r}"


def test_multi_broadcast_and_info(ctx):
    dev = torch.device("cuda", 0)
    t = torch.arange(1000, dtype=torch.float64, device=dev)
    ref = t.clone()
    ctx.broadcast([t.data_ptr()], t.numel() * 8, 0)
    assert torch.equal(t, ref)
    assert (ctx.world, ctx.n_local, ctx.first_rank) == (1, 1, 0)


def test_multi_errors(ctx, orc):
    rp, ci, v = orc.gen_csr(1000, 100, 50, 1, 0, 5)
    ci_bad = ci.copy()
    if ci_bad.size:
        ci_bad[ci_bad.size // 2] = 50  # column == cols: the reference's index panic (sparse.rs:437)
    with pytest.raises(_lib.BsmError) as e:
        MultiCsr.upload(ctx, 100, 50, rp, ci_bad, v, chunks=2)
    assert e.value.code == _lib.BSM_ERR_PANIC
    m = MultiCsr.upload(ctx, 100, 50, rp, ci, v)
    with pytest.raises(_lib.BsmError) as e:
        m.mul_dense_cols(orc.gen_x_cols(1001, 49, 2), 49)
    assert e.value.code == _lib.BSM_ERR_DIMENSIONS
    with pytest.raises(_lib.BsmError):
        MultiGpu(64)  # more GPUs than visible


def test_public_api_over_set_gpus(orc):
    """The mirror's Csr.mul_dense routed over the row-block path on one GPU
    (what a Rust mul_dense does once its context has n GPUs)."""
    rp, ci, v = orc.gen_csr(1000, 4000, 4000, 1, 0, 30)
    x_cols = orc.gen_x_cols(1001, 4000, 32)
    a = Csr.from_csr_arrays((4000, 4000), rp, ci, v)
    try:
        bsm.set_gpus(1, chunks=3)
        got = a.mul_dense(Dense.from_columns(x_cols))
        got2 = a.mul_dense(Dense.from_columns(x_cols))  # the cached partition
    finally:
        bsm.set_gpus(None)
    want = orc.mul_dense(4000, 4000, rp, ci, v, x_cols)
    assert_same_csr((got.row_index, got.col_index, got.v), want)
    assert_same_csr((got2.row_index, got2.col_index, got2.v), want)
    with pytest.raises(Panic):
        bsm.set_gpus(1)
        try:
            Csr.from_csr_arrays((2, 2), np.array([0, 1, 2], np.uint64), np.array([0, 5], np.uint64),
                                np.array([1.0, 2.0])).mul_dense(Dense.from_columns([np.ones(2)]))
        finally:
            bsm.set_gpus(None)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("chunks", [1, 3])
def test_bench_under_torchrun_nccl(chunks):
    """bench.py --gpus 1 as a fresh torch.distributed.run job, backend nccl:
    the library's RCCL context from a shipped id, its all-gathers, torch's
    RCCL barrier / all-reduce, and --verify (bit-identical to one GPU)."""
    env = dict(os.environ, BSM_MULTI_SOLO_RCCL="1")
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "1", "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(ROOT, "bench.py"), "--gpus", "1",
           "--config", "c3", "--steps", "3", "--warmup", "1", "--no-cpu-baseline", "--no-e2e", "--verify",
           "--chunks", str(chunks), "--backend", "nccl"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["verified_vs_single_gpu"] is True and line["verified_rows"] == 1_000_000
    assert "RCCL" in line["config"]["comm"] and "nccl" in line["config"]["comm"]
    assert line["n_gpus"] == 1 and line["value"] > 0


def test_multi_skewed_rows_pieces_capped(ctx, orc):
    """nnz-balanced pieces on a matrix with a long run of empty rows
    gave one piece nearly every row, and every device P x the single-GPU Y.
    The cost split (a row costs its entries + max(1, nnz/rows)) caps a piece
    at 2*rows/P + 1 rows; the product stays bit-exact."""
    rows, cols, k, chunks = 10_000, 3000, 32, 4
    lens = np.concatenate([np.zeros(9000, np.int64), np.full(1000, 60)])
    rp = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    rng = np.random.default_rng(3)
    ci = np.concatenate([np.sort(rng.choice(cols, 60, replace=False)) for _ in range(1000)]).astype(np.uint64)
    v = rng.uniform(0.5, 1.5, ci.size)
    x_cols = orc.gen_x_cols(1001, cols, k)
    m = MultiCsr.upload(ctx, rows, cols, rp, ci, v, chunks=chunks)
    assert m.piece_rows <= 2 * rows / chunks + 1, m.piece_rows
    assert_same_csr(m.mul_dense_cols(x_cols, cols).download(), orc.mul_dense(rows, cols, rp, ci, v, x_cols))


def test_multi_concurrent_calls_one_matrix(ctx, orc):
    """calls on one bsm_mcsr from several threads (a cached
    partition reached from &self) are serialised by the handle's lock; with
    different k each call re-prepares, so without it one call would free the
    buffers under the other."""
    import threading

    rows, cols = 3000, 2000
    rp, ci, v = orc.gen_csr(1000, rows, cols, 1, 0, 30)
    m = MultiCsr.upload(ctx, rows, cols, rp, ci, v, chunks=2)
    xs = {k: orc.gen_x_cols(1001, cols, k) for k in (1, 8, 32)}
    want = {k: orc.mul_dense(rows, cols, rp, ci, v, x) for k, x in xs.items()}
    errors = []

    def run(k):
        try:
            for _ in range(4):
                assert_same_csr(m.mul_dense_cols(xs[k], cols).download(), want[k])
        except Exception as e:  # noqa: BLE001
            errors.append((k, repr(e)))

    th = [threading.Thread(target=run, args=(k,)) for k in (1, 8, 32, 8)]
    for t in th:
        t.start()
    for t in th:
        t.join(120)
    assert not errors, errors


def test_external_context_world1_and_refusals(orc):
    """bsm_multi_create_external at world 1: step fills every slot itself; the
    exchange is a no-op, compact builds the output. mul_dense and broadcast
    need a communicator and say so."""
    c = MultiGpu.external(1, 0, 0)
    assert c.is_external
    rows, cols, k = 2000, 3000, 32
    rp, ci, v = orc.gen_csr(1000, rows, cols, 1, 0, 30)
    x_cols = orc.gen_x_cols(1001, cols, k)
    m = MultiCsr.upload(c, rows, cols, rp, ci, v, chunks=3)
    m.prepare(k)
    x = torch.from_numpy(np.ascontiguousarray(np.stack(x_cols, axis=1))).cuda()
    m.step([x.data_ptr()])
    m.sync()
    y, nz = m.slot_read(0, m.pieces)
    assert y.shape == (m.pieces, m.piece_rows, k)
    m.slot_write(0, y, nz)  # round trip
    m.compact()
    m.sync()
    assert_same_csr(m.output().download(), orc.mul_dense(rows, cols, rp, ci, v, x_cols))
    with pytest.raises(_lib.BsmError) as e:
        m.mul_dense_cols(x_cols, cols)
    assert e.value.code == _lib.BSM_ERR_UNSUPPORTED
    with pytest.raises(_lib.BsmError) as e:
        c.broadcast([x.data_ptr()], 8, 0)
    assert e.value.code == _lib.BSM_ERR_UNSUPPORTED
    with pytest.raises(_lib.BsmError):
        m.slot_read(m.pieces, 1)  # past the last slot
    del m
    c.close()


@pytest.mark.parametrize("chunks", [1, 3])
def test_one_rank_skips_allgathers_same_bits(ctx, orc, monkeypatch, chunks):
    """One rank: the default step skips the degenerate all-gathers and their
    stream hops; the output is the same as with them (BSM_MULTI_SOLO_RCCL=1)."""
    rows, cols, k = 3000, 2000, 32
    rp, ci, v = orc.gen_csr(1000, rows, cols, 1, 0, 40)
    x_cols = orc.gen_x_cols(1001, cols, k)
    m = MultiCsr.upload(ctx, rows, cols, rp, ci, v, chunks=chunks)
    monkeypatch.setenv("BSM_MULTI_SOLO_RCCL", "0")
    skipped = m.mul_dense_cols(x_cols, cols).download()
    monkeypatch.setenv("BSM_MULTI_SOLO_RCCL", "1")
    with_rccl = m.mul_dense_cols(x_cols, cols).download()
    assert_same_csr(skipped, with_rccl)
    assert_same_csr(skipped, orc.mul_dense(rows, cols, rp, ci, v, x_cols))
