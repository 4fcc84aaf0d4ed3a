"""The multi-rank SpMM path (BASELINE.json north_star config 4: rows
partitioned across GPUs, RHS replicated, Y all-gathered) run
on the GPU: 2 and 3 ranks as fresh child processes (gloo, all on cuda:0),
each running the HIP SpMM on its block-cyclic row pieces exactly as
bench.py's step does. The assembled Y and per-row counts must be bit-identical
to the single-GPU product, and the compacted Csr equal to the CPU oracle on a
sampled row range (rows are independent in src/sparse.rs:431-444).
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


@pytest.mark.parametrize("world,rows,n_cols,nnz_r,k,chunks,panel", [
    (2, 20_011, 5_000, 12, 32, 3, 0),     # k = 32 rows kernel, clipped last round
    (2, 20_011, 5_000, 12, 32, 3, 350),   # column-panel plan (15 panels of 350 columns)
    (3, 9_001, 3_000, 6, 1, 3, 0),        # SpMV arm (k = 1)
    (2, 4_099, 4_000, 40, 7, 3, 0),       # general-k kernel
    (2, 20_011, 5_000, 12, 32, 3, -1),    # tiled copy per piece (k = 32), several batches: the batch pacing
    (3, 9_001, 3_000, 6, 1, 2, -1),       # tiled copy, k = 1   barrier with two grids sharing the CUs
])
def test_block_cyclic_spmm_on_gpu_matches_single(tmp_path, world, rows, n_cols, nnz_r, k, chunks, panel):
    port = _free_port()
    outs = [tmp_path / f"rank{r}.json" for r in range(world)]
    procs = []
    for r in range(world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(world), LOCAL_RANK=str(r),
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
        if panel == -1:  # small batches so the pacing barrier is live
            env.update(BSM_TILED_RW="64" if k == 32 else "40", BSM_TILED_WAVES="16")
        procs.append(subprocess.Popen([sys.executable, "-u", WORKER, str(outs[r]), str(rows), str(n_cols),
                                       str(nnz_r), str(k), str(chunks), str(panel)], env=env,
                                      stdout=subprocess.PIPE, stderr=subprocess.STDOUT))
    logs = []
    try:
        for p in procs:
            out, _ = p.communicate(timeout=100)
            logs.append(out.decode(errors="replace")[-2000:])
    finally:
        for p in procs:
            if p.poll() is None:
                p.kill()
    assert all(p.returncode == 0 for p in procs), logs
    res = json.loads(outs[0].read_text())
    if panel == -1:
        assert any(w == -1 for w in res["widths"]), res  # the tiled kernel really ran
    elif panel:
        assert all(w == panel for w in res["widths"]), res  # the panelled kernel really ran
    assert res["y_equal"] and res["nnz_equal"], res
    assert res["oracle_equal"], res
