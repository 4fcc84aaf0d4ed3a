"""The library's multi-GPU Csr::mul_dense at world 2, 3 and 8 (BASELINE.json
north_star / configs[3]: rows partitioned across GPUs, X replicated, Y
assembled) on the one GPU of the box.

Each rank is a fresh process on cuda:0 with an external context
(bsm_multi_create_external: RCCL allows one rank per device, so the slots of
the gathered Y move over gloo instead of ncclAllGather; see
tests/dist_spmm_worker.py). Everything else is the library's own multi-GPU
code: the piece bounds, round c of rank r in slot c*world + r, the slot
padding, the row_ptr squeeze over short pieces, empty pieces, the tiled and
panelled schedules per piece, and the compaction. Rows are independent in
the reference (src/sparse.rs:431-444), so the output Csr of every rank must
be bit-identical to the single-GPU bsm_csr_mul_dense and to the oracle.
"""

import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

HERE = os.path.dirname(os.path.abspath(__file__))
WORKER = os.path.join(HERE, "dist_spmm_worker.py")


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _run(tmp_path, world, args, env_extra=None, timeout=100):
    port = _free_port()
    outs = [tmp_path / f"rank{r}.json" for r in range(world)]
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r), MASTER_ADDR="127.0.0.1",
                   MASTER_PORT=str(port))
        env.update(env_extra or {})
        procs.append(subprocess.Popen([sys.executable, "-u", WORKER, str(outs[r])] + [str(a) for a in args], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    logs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=timeout)
            logs.append(out.decode(errors="replace")[-2000:])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert all(p.returncode == 0 for p in procs), logs
    return [json.loads(o.read_text()) for o in outs]


# rows, n_cols, kind, a, b, k, chunks, schedule, dtype
UPLOAD_CASES = [
    (2, 3000, 2000, 1, 0, 40, 32, 1, "auto", "f64"),   # uneven pieces: squeeze
    (2, 3000, 2000, 1, 0, 40, 32, 3, "auto", "f64"),
    (3, 3000, 2000, 1, 0, 40, 32, 1, "auto", "f64"),
    (3, 3001, 2000, 1, 0, 40, 32, 3, "panel", "f64"),
    (3, 2000, 3000, 0, 20, 20, 32, 3, "auto", "f64"),  # equal pieces: no squeeze
    (2, 1000, 5000, 1, 0, 7, 1, 3, "auto", "f64"),     # SpMV arm
    (3, 777, 513, 1, 0, 20, 5, 2, "auto", "f32"),      # general k, f32
    (2, 500, 400, 1, 1, 9, 3, 3, "auto", "i32"),       # integer (wrapping) sums
    (3, 10, 30, 1, 0, 12, 2, 4, "auto", "f64"),        # 12 pieces for 10 rows: empty pieces
    (2, 64, 64, 1, 0, 3, 0, 2, "auto", "f64"),         # k = 0: every output row empty
    # world 8, north_star's split (configs[3]): 8 or 16 pieces
    (8, 3000, 2000, 1, 0, 40, 32, 1, "auto", "f64"),   # uneven pieces: squeeze across 8
    (8, 3001, 2000, 1, 0, 40, 32, 2, "panel", "f64"),  # 16 pieces, slot offsets up to 15 pad k
    (8, 2000, 3000, 0, 20, 20, 32, 2, "auto", "f64"),  # equal pieces
    (8, 1000, 5000, 1, 0, 7, 1, 2, "auto", "f64"),     # SpMV arm
    (8, 10, 30, 1, 0, 12, 2, 2, "auto", "f64"),        # 16 pieces for 10 rows: empty pieces
]


@pytest.mark.parametrize("world,rows,n_cols,kind,a,b,k,chunks,schedule,dtype", UPLOAD_CASES)
def test_external_ranks_upload_match_single_and_oracle(tmp_path, world, rows, n_cols, kind, a, b, k, chunks,
                                                       schedule, dtype):
    res = _run(tmp_path, world, ["upload", rows, n_cols, kind, a, b, k, chunks, schedule, dtype],
               timeout=100 if world < 8 else 240)
    r0 = res[0]
    assert r0["pieces"] == world * chunks
    assert all(r["ranks_agree"] and r["steps_equal"] and r["bounds_equal_mirror"] for r in res), res
    assert r0["oracle_equal"] and r0["single_equal"], r0
    if rows == 10:
        assert r0["empty_pieces"] > 0
    if kind == 1 and rows >= 1000:
        assert r0["squeeze"], r0  # short pieces before the last: the row_ptr squeeze ran


GEN_CASES = [
    # tiled copy per piece (forced), small batches so the pacing barrier is live
    # with two or three grids sharing the CUs
    (2, 20_011, 5_000, 1, 0, 24, 32, 1, "tiled"),
    (3, 20_011, 5_000, 1, 0, 24, 32, 3, "tiled"),
    (3, 9_001, 3_000, 1, 0, 12, 1, 2, "tiled"),       # tiled k = 1
    (2, 20_011, 30_000, 1, 0, 24, 32, 3, "panel"),    # never the copy
    (8, 20_011, 5_000, 1, 0, 24, 32, 1, "tiled"),     # world 8: 8 grids share the CUs
    (8, 20_011, 5_000, 1, 0, 24, 32, 2, "tiled"),
    (8, 20_011, 30_000, 1, 0, 24, 32, 2, "panel"),
    # a C4-shaped block (10M columns, 1000 nnz/row, k = 32) at world 8 with
    # the library's default schedule and geometry (the tiled copy per piece)
    (8, 1_000_000, 10_000_000, 0, 1000, 1000, 32, 1, "auto"),
    (8, 1_000_000, 10_000_000, 0, 1000, 1000, 32, 2, "auto"),
]


@pytest.mark.parametrize("world,rows,n_cols,kind,a,b,k,chunks,schedule", GEN_CASES)
def test_external_ranks_generate_schedules(tmp_path, world, rows, n_cols, kind, a, b, k, chunks, schedule):
    env = {"BSM_TILED_RW": "64" if k == 32 else "40", "BSM_TILED_WAVES": "16"} if schedule == "tiled" else {}
    res = _run(tmp_path, world, ["generate", rows, n_cols, kind, a, b, k, chunks, schedule, "f64"], env,
               timeout=100 if world < 8 else 300)
    r0 = res[0]
    assert all(r["ranks_agree"] and r["steps_equal"] for r in res), res
    assert r0["single_equal"] and r0["oracle_equal"], r0
    for r in res:
        assert r["plan"]["local_pieces"] == chunks
        if schedule == "tiled" or n_cols >= 10_000_000:
            assert r["plan"]["tiled_pieces"] == chunks, r  # the copy really ran on every piece
        else:
            assert r["plan"]["tiled_pieces"] == 0, r


@pytest.mark.parametrize("world,out_rank", [(3, 0), (8, 5)])
def test_external_ranks_single_output_rank(tmp_path, world, out_rank):
    """bsm_mcsr_set_output_rank: only one rank compacts the gathered Y and
    returns the output Csr (the other ranks hold no output buffers and refuse
    bsm_mcsr_output); that Csr is the single-GPU one and the oracle's."""
    res = _run(tmp_path, world, ["upload", 3000, 2000, 1, 0, 40, 32, 2, "auto", "f64"],
               {"DIST_OUTPUT_RANK": str(out_rank)}, timeout=100 if world < 8 else 240)
    assert all(r["ranks_agree"] and r["steps_equal"] for r in res), res
    r = res[out_rank]
    assert r["oracle_equal"] and r["single_equal"], r


@pytest.mark.parametrize("config,chunks,world", [("c3", 1, 2), ("c3", 3, 2), ("c3", 1, 8), ("c3", 2, 8)])
def test_bench_ranks_one_gpu_gloo_exchange(config, chunks, world):
    """bench.py's N > 1 path (the rank's pieces, my_rows, the barriers, the
    max over ranks, --verify of the assembled Y against one GPU, the JSON
    line) with two or eight ranks on the one GPU: external contexts, Y slots over gloo
    (--exchange gloo). A logic check of what the driver's N = 2..8 runs do
    with RCCL, not a measurement."""
    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    root = os.path.dirname(HERE)
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", str(world), "--master-addr",
           "127.0.0.1", "--master-port", str(_free_port()), os.path.join(root, "bench.py"), "--gpus", str(world),
           "--config", config, "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--no-e2e", "--verify",
           "--chunks", str(chunks), "--exchange", "gloo"]
    r = subprocess.run(cmd, capture_output=True, text=True, timeout=300, env=env, cwd=root)
    assert r.returncode == 0, r.stdout[-3000:] + r.stderr[-3000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == world and line["verified_vs_single_gpu"] is True
    assert line["verified_rows"] == 1_000_000
    assert "external" in line["config"]["comm"]
