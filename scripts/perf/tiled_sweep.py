"""Sweep the row-block x column-panel schedule's geometry on the C4 shape
(or a leading row fraction of it) in one process: for each variant
(env BSM_TILED_* read at plan creation) build the copy, time the SpMM with
HIP events and print one line. Also times the one-pass/panelled kernel for
reference. Usage: python scripts/perf/tiled_sweep.py [rows] VAR=VAL,VAR=VAL ..."""

import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402

from basic_sparse_matrix_amd import _lib  # noqa: E402
from basic_sparse_matrix_amd.device import DeviceCsrBlock, gen_dense  # noqa: E402


def timed(fn, reps=3):
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    fn()
    torch.cuda.synchronize()
    ts = []
    for _ in range(reps):
        e0.record()
        fn()
        e1.record()
        torch.cuda.synchronize()
        ts.append(e0.elapsed_time(e1))
    return min(ts), float(np.mean(ts))


def main():
    rows = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
    variants = sys.argv[2:] or [""]
    c2 = os.environ.get("SWEEP_SHAPE") == "c2"  # C2: 1M x 1M, 10 nnz/row, k = 1
    n_cols, k, nnz_r = (1_000_000, 1, 10) if c2 else (10_000_000, 32, 1000)
    torch.cuda.set_device(0)
    t0 = time.perf_counter()
    blk = DeviceCsrBlock.generate(1000, 0, rows, n_cols, _lib.ROWLEN_CONST, nnz_r, nnz_r)
    x = gen_dense(1001, 0, n_cols, k)
    y = torch.empty((rows, k), dtype=torch.float64, device="cuda")
    nnz = torch.empty(rows, dtype=torch.int32, device="cuda")
    torch.cuda.synchronize()
    scale = (1_000_000 if c2 else 10_000_000) / rows
    print(f"generated {rows:,} rows in {time.perf_counter() - t0:.1f} s", flush=True)
    ref = None
    if os.environ.get("SWEEP_REF", "1") == "1":
        blk.plan(k)
        best, mean = timed(lambda: blk.spmm(x, y, nnz), reps=20 if c2 else 3)
        ref = y.clone()
        print(f"untiled ({blk.panel_cols} panel cols): {best:.3f} ms (mean {mean:.3f}), scaled {best * scale:.3f} ms",
              flush=True)
        blk.seg, blk.panel_cols = None, 0
    for var in variants:
        env = dict(kv.split("=") for kv in var.split(",") if kv)
        saved = {kk: os.environ.get(kk) for kk in env}
        os.environ.update(env)
        t0 = time.perf_counter()
        plan = blk.plan_tiled(k, force=True)
        torch.cuda.synchronize()
        build_ms = (time.perf_counter() - t0) * 1e3
        for kk, vv in saved.items():
            if vv is None:
                os.environ.pop(kk, None)
            else:
                os.environ[kk] = vv
        if plan is None:
            print(f"{var or 'default'}: declined", flush=True)
            continue
        info = plan.info()
        best, mean = timed(lambda: blk.spmm(x, y, nnz), reps=20 if c2 else 3)
        same = None if ref is None else bool(torch.equal(y.view(torch.int64), ref.view(torch.int64)))
        print(f"{var or 'default'}: {best:.3f} ms (mean {mean:.3f}), scaled {best * scale:.3f} ms, "
              f"gather {rows * nnz_r * 8 * k / best / 1e9:.2f} TB/s, padding {info['slots'] / blk.nnz - 1:.4f}, "
              f"build {build_ms:.0f} ms, same bits {same}", flush=True)
        blk.tiled = None
        del plan
        torch.cuda.synchronize()


if __name__ == "__main__":
    main()
