#!/usr/bin/env python3
"""bench.py -- CSR x dense SpMM throughput on MI355X (BASELINE.json metric:
"CSR x dense SpMM effective GB/s (% HBM3E peak) at 1/2/4/8 GPUs; nnz/s").

Workload (BASELINE.json north_star target / configs[3]): A = 10M x 10M
synthetic random CSR, 1000 nnz per row (0.01 % density, nnz = 1e10), f64,
times a dense 10M x 32 f64 RHS. It fits one MI355X (A 120 GB + X/Y 5 GB of
288 GB HBM), so N=1 runs the whole matrix on one GPU. For N > 1 the rows are
split block-cyclically (one process per GPU): `--chunks` rounds of N equal
row blocks, rank g owning block g of every round (equal rows = equal nnz). X
is replicated (every rank generates the same X from its seed -- no transfer)
and the dense result Y is assembled on every rank with RCCL all-gathers over
xGMI, as north_star specifies: one async all-gather per round, issued as soon
as that round's SpMM is enqueued, so it overlaps the next round's SpMM and
lands in global row order. Total work is fixed as N grows ("strong").

One step = the hot path of Csr::mul_dense (src/sparse.rs:426-446) over the
whole matrix: SpMM kernel (Y block) -> [all-gather of Y blocks] ->
compaction of Y into the output Csr (zero-dropping insert, sparse.rs:229).
Inputs are resident in HBM before timing starts.

value = B_alg / step time (whole job), with the canonical algorithmic bytes
of SURVEY.md §8d: B_alg = 8(N+1) + 12 nnz + 8 n_cols k + 8 N k.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

import numpy as np  # noqa: E402
import torch  # noqa: E402  (imported before the HIP library: one runtime)
import torch.distributed as dist  # noqa: E402

CONFIGS = {
    # name: (rows, n_cols, nnz_per_row, k); BASELINE.json configs[0..3]
    "c4": (10_000_000, 10_000_000, 1000, 32),
    "c3": (1_000_000, 1_000_000, 10, 32),
    "c2": (1_000_000, 1_000_000, 10, 1),
    "c1": (1024, 1024, None, 1),  # row lengths ~ Binomial(1024, 0.01): ~10.5k nnz (host generator)
}
C1_P = 0.01
HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md)
ROWLEN_CONST, ROWLEN_BINOMIAL = 0, 2  # bsm_synth.h row-length families
SEED_A, SEED_X = 1000, 1001


def b_alg(rows, n_cols, nnz, k):
    return 8 * (rows + 1) + 12 * nnz + 8 * n_cols * k + 8 * rows * k


def b_gather(rows, nnz, k):
    """SURVEY.md §8d traffic model: every nnz gathers its whole X row (no reuse
    beyond the caches): 8(N+1) + 12 nnz + 8 nnz k + 8 N k."""
    return 8 * (rows + 1) + 12 * nnz + 8 * nnz * k + 8 * rows * k


def kernel_label(rows, nnz, k, panel_cols, tiled=False):
    """The kernel launch_spmm (kernels_spmm.hip) picks for this shape."""
    if tiled:
        return f"spmm_tiled_k{k}"
    if k == 1:
        if nnz <= 12 * rows:
            return "spmv_wave<double,8>"
        return "spmv_stream<double,4>"
    if k == 32:
        if nnz <= 24 * rows and not panel_cols:
            return "spmm_k32_f64_rows4<4>"
        return f"spmm_k32_f64<4,true,{'true' if panel_cols else 'false'}>"
    return "spmm_rowwave<double>"


def end_to_end(cfg_name, blks, x, comp, step, rows, k, iters=3):
    """End-to-end figures next to the device-resident step:
    device_ms = H2D of X from pinned host memory + the step + D2H of the
    output Csr (row_ptr, col, vals) into pinned host memory, A resident (as the
    host mirror caches it); public_api_ms (host-sized configs only) =
    Csr.mul_dense(Dense) through the public API, host Dense in, host Csr out
    (the library's own X upload/packing and int32 -> usize column widening)."""
    out = {}
    n_out = comp.nnz()
    xh = x.cpu().pin_memory()
    rp_h = torch.empty(rows + 1, dtype=torch.int64).pin_memory()
    col_h = torch.empty(max(1, n_out), dtype=torch.int32).pin_memory()
    val_h = torch.empty(max(1, n_out), dtype=torch.float64).pin_memory()
    ts = []
    for _ in range(iters):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        x.copy_(xh, non_blocking=True)
        step(False)
        rp_h.copy_(comp.row_ptr, non_blocking=True)
        col_h[:n_out].copy_(comp.col[:n_out], non_blocking=True)
        val_h[:n_out].copy_(comp.vals[:n_out], non_blocking=True)
        torch.cuda.synchronize()
        ts.append(time.perf_counter() - t0)
    out["device_ms"] = round(float(np.median(ts)) * 1e3, 3)
    out["h2d_bytes"] = int(xh.numel() * 8)
    out["d2h_bytes"] = int((rows + 1) * 8 + n_out * 12)
    if len(blks) == 1 and blks[0].nnz <= 200_000_000:
        from basic_sparse_matrix_amd import Csr, Dense

        b = blks[0]
        a = Csr.from_csr_arrays((b.rows, b.n_cols), b.row_ptr.cpu().numpy().astype(np.uint64),
                                b.col.cpu().numpy().astype(np.uint64), b.vals.cpu().numpy())
        xd = Dense.from_columns([np.ascontiguousarray(xh[:, j].numpy()) for j in range(k)])
        a.mul_dense(xd)  # first call uploads and caches A on the device (untimed, like the bench's setup)
        ts = []
        for _ in range(max(iters, 20 if cfg_name == "c1" else iters)):
            t0 = time.perf_counter()
            a.mul_dense(xd)
            ts.append(time.perf_counter() - t0)
        out["public_api_ms"] = round(float(np.median(ts)) * 1e3, 4)
        out["public_api_calls"] = len(ts)
    return out


def log(msg):
    print(f"[bench] {msg}", file=sys.stderr, flush=True)


def c1_rowlen_a():
    """Binomial(1024, p) row lengths: p = a / 2^32 (bsm_synth.h bsm_rowlen_binomial)."""
    return int(round(C1_P * 2 ** 32))


def rowlen_spec(cfg_name):
    """(kind, a, b) of the synthetic row-length family of a config."""
    rows, n_cols, nnz_r, k = CONFIGS[cfg_name]
    if nnz_r is None:
        return ROWLEN_BINOMIAL, c1_rowlen_a(), 0
    return ROWLEN_CONST, nnz_r, nnz_r


def cpu_baseline(cfg_name, sample_rows, reps=20):
    """The oracle's restatement of Csr::mul_dense (oracle/, single thread),
    with get_row_compact's per-row Vec allocation emulated
    (orc_set_emulate_row_alloc). A config that fits (C1-C3 row counts up to
    `sample_rows`) is timed whole, median of `reps` calls; a bigger one (C4)
    on its first `sample_rows` rows, extrapolated linearly to the full row
    count (its rows are statistically identical)."""
    from oracle import pyoracle as orc

    rows, n_cols, _, k = CONFIGS[cfg_name]
    kind, a, b = rowlen_spec(cfg_name)
    n = min(rows, sample_rows)
    rp = orc.gen_row_ptr(SEED_A, n, n_cols, kind, a, b)
    ci, v = orc.gen_entries(SEED_A, rp, n_cols)
    t0 = time.perf_counter()
    x_cols = orc.gen_x_cols(SEED_X, n_cols, k)
    t_gen = time.perf_counter() - t0
    orc.lib().orc_set_emulate_row_alloc(1)
    try:
        ts = []
        while True:  # whole matrix: `reps` calls, fewer if they would take over ~30 s
            t0 = time.perf_counter()
            orc.mul_dense(n, n_cols, rp, ci, v, x_cols)
            ts.append(time.perf_counter() - t0)
            if n < rows or len(ts) >= reps or (len(ts) >= 3 and sum(ts) > 30.0):
                break
    finally:
        orc.lib().orc_set_emulate_row_alloc(0)
    t = float(np.median(ts))
    t_full = t * rows / n
    nnz_s = int(rp[n])
    nnz = nnz_s if n == rows else nnz_s * rows // n
    how = (f"whole matrix, median of {len(ts)} calls ({t * 1e3:.3f} ms)" if n == rows else
           f"first {n} of {rows} rows ({nnz_s} nnz x {k} RHS) in {t:.2f} s, extrapolated x{rows // n} "
           f"to {t_full:.1f} s per full SpMM")
    return {
        "value": round(b_alg(rows, n_cols, nnz, k) / t_full / 1e9, 4),
        "unit": "GB/s",
        "cores": 1,
        "kind": "port",
        "sample": f"oracle mul_dense (C restatement of sparse.rs:426-446, -O2 -ffp-contract=off, 1 thread, "
                  f"get_row_compact's per-row dims.cols x 24 B Vec allocated as in sparse.rs:254; output "
                  f"arrays preallocated, where the reference grows Vecs) on the {how} (X generation "
                  f"{t_gen:.1f} s untimed)",
        "ms_per_spmm": round(t_full * 1e3, 4),
        "nnz_per_s": round(nnz_s / t, 1),
        "host_cpus": os.cpu_count(),
    }


def bench_x_cols(seed, k, n, fill, dtype=np.uint32):
    """The reference bench's RHS (sparse_dense_mul.rs:23-29): k zero columns of
    n, then `fill` writes of v % 255 at (col % k, row % n); later writes win."""
    rng = np.random.default_rng(seed)
    cols = [np.zeros(n, dtype=dtype) for _ in range(k)]
    j = rng.integers(0, k, fill)
    i = rng.integers(0, n, fill)
    v = rng.integers(0, 255, fill)
    for a, b, c in zip(j, i, v):
        cols[a][b] = c
    return cols


def _time_call(fn, iters, warm=3):
    for _ in range(warm):
        out = fn()
    ts = []
    for _ in range(iters):
        t0 = time.perf_counter()
        out = fn()
        ts.append(time.perf_counter() - t0)
    return out, float(np.median(ts))


def _same(out, ref):
    e_rp, e_ci, e_v = ref
    return bool(np.array_equal(np.asarray(out.row_index, np.uint64), e_rp)
                and np.array_equal(np.asarray(out.col_index, np.uint64), e_ci)
                and np.array_equal(np.asarray(out.v), e_v))


def ref_bench_suite(iters=20, which=("sd_mul", "ss_add", "ss_mul")):
    """The reference's own criterion benches, one JSON line per size:
      sd_mul (sparse_dense_mul.rs:6-35): Csr<u32> 1000 x 1000 from e random
        inserts x a 10-column Dense<u32> with e/100 random entries;
      ss_add (sparse_dense_mul.rs:37-67): two such Csr<u32>, add_sparse;
      ss_mul (sparse_sparse_mul.rs:6-37): two such Csr<u32>, mul_sparse.
    criterion's throughput unit is elements = e per call. GPU: the public
    Csr call end to end (uploads, kernels, download), the matrices built on
    the device by the insert-sequence builder. CPU: the oracle's restatement
    of the same call (1 thread) on the same inputs, which is also the check
    (bit_exact_vs_oracle). The insert streams come from bsm_synth.h's
    SplitMix64 (StdRng is not vendored), with the benches' shapes."""
    from basic_sparse_matrix_amd import Dense
    from basic_sparse_matrix_amd.device import csr_from_device_inserts, gen_insert_stream
    from oracle import pyoracle as orc

    def build(seed, e):
        r, c, v = gen_insert_stream(seed, e, 1000, 1000, 255, np.uint32)
        return csr_from_device_inserts((1000, 1000), r, c, v)

    def arrays(m):
        return (1000, 1000, np.asarray(m.row_index, np.uint64), np.asarray(m.col_index, np.uint64),
                np.asarray(m.v))

    sizes = {
        "sd_mul": [10000 * (i + 1) * 10 for i in range(9)],
        "ss_add": [10000 * (i + 1) * 10 for i in range(9)],
        "ss_mul": [i * 50 for i in [1, 2, 5, 10, 20, 50, 100, 200, 500, 1000, 2000, 10000]],
    }
    cite = {"sd_mul": "benches/sparse_dense_mul.rs:6-35", "ss_add": "benches/sparse_dense_mul.rs:37-67",
            "ss_mul": "benches/sparse_sparse_mul.rs:6-37"}
    for name in which:
        for e in sizes[name]:
            a = build(SEED_A, e)
            if name == "sd_mul":
                x_cols = bench_x_cols(SEED_X + e, 10, 1000, e // 100)
                x = Dense.from_columns(x_cols)
                out, gpu_s = _time_call(lambda: a.mul_dense(x), iters)
                ra = arrays(a)
                cpu = lambda: orc.mul_dense(1000, 1000, ra[2], ra[3], ra[4], x_cols)  # noqa: E731
                extra = {"k": 10, "longest_row": int(np.diff(ra[2].astype(np.int64)).max())}
            else:
                b = build(SEED_X, e)
                op = a.add_sparse if name == "ss_add" else a.mul_sparse
                out, gpu_s = _time_call(lambda: op(b), iters if name == "ss_add" or e <= 100_000 else 5)
                ra, rb = arrays(a), arrays(b)
                cpu_fn = orc.add_sparse if name == "ss_add" else orc.mul_sparse
                cpu = lambda: cpu_fn(ra, rb)  # noqa: E731
                extra = {"b_nnz": int(b.get_nnz())}
            cts = []
            for _ in range(3 if name != "ss_mul" or e <= 100_000 else 1):
                t0 = time.perf_counter()
                ref = cpu()
                cts.append(time.perf_counter() - t0)
            cpu_s = float(np.median(cts))
            print(json.dumps({
                "workload": f"{name} ({cite[name]})", "elements": e, "dtype": "u32", "a_nnz": int(a.get_nnz()),
                **extra, "gpu_ms_per_call": round(gpu_s * 1e3, 4), "gpu_elements_per_s": round(e / gpu_s, 1),
                "cpu_ms_per_call": round(cpu_s * 1e3, 4), "cpu_elements_per_s": round(e / cpu_s, 1),
                "cpu_kind": "port (oracle restatement, 1 thread)", "gpu_over_cpu": round(cpu_s / gpu_s, 2),
                "out_nnz": int(out.get_nnz()), "bit_exact_vs_oracle": _same(out, ref),
            }), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-rows", type=int, default=100_000,
                    help="rows of the CPU baseline sample (configs with more rows are extrapolated)")
    ap.add_argument("--panel-cols", type=int, default=None,
                    help="column-panel width of the SpMM schedule (default: the library's choice; 0 = one pass)")
    ap.add_argument("--schedule", default="auto", choices=("auto", "tiled", "panel"),
                    help="SpMM schedule: auto = the library's choice (row-block x column-panel copy when "
                         "wanted, else column panels), tiled = the copy whenever possible, panel = never the copy")
    ap.add_argument("--chunks", type=int, default=0,
                    help="rounds of the block-cyclic row partition (0: 1 at N=1, 4 at N>1)")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for N > 1 (nccl = RCCL)")
    ap.add_argument("--verify", action="store_true",
                    help="rank 0 recomputes the whole Y on its own GPU and checks the assembled Y bit for bit")
    ap.add_argument("--traffic-bytes", type=float, default=None,
                    help="PMC-measured HBM bytes per SpMM launch (from profiles/), reported as roofline.traffic")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (H2D/D2H included) figures")
    ap.add_argument("--ref-benches", default=None,
                    help="comma list of the reference's own criterion benches to run instead "
                         "(sd_mul,ss_add,ss_mul; one JSON line per size)")
    args = ap.parse_args()
    if args.ref_benches:
        ref_bench_suite(which=tuple(args.ref_benches.split(",")))
        return

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")
    # one GPU per rank; ranks beyond the visible GPUs share them (rehearsals)
    ordinal = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(ordinal)
    dev = torch.device("cuda", ordinal)
    if world > 1:
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(args.backend)

    from basic_sparse_matrix_amd import _lib
    from basic_sparse_matrix_amd.device import Compactor, DeviceCsrBlock, gen_dense

    from basic_sparse_matrix_amd.distributed import partition_rows_cyclic

    rows, n_cols, nnz_r, k = CONFIGS[args.config]
    kind, ra, rb = rowlen_spec(args.config)
    # block-cyclic row partition (equal rows = equal nnz: constant row length):
    # `chunks` rounds, each finished by its own SpMM launch and all-gathered
    # asynchronously while the next round computes (N > 1)
    # one round per rank when the tiled copy serves the shape: its persistent
    # grid wants every CU (an all-gather kernel beside it would hold some and
    # defeat its batch pacing), so the all-gather follows the SpMM instead of
    # overlapping a next round
    lib0 = _lib.load()
    tiled_shape = args.schedule != "panel" and k in (1, 32) and bool(lib0.bsm_dev_tiled_wanted(
        _lib.DTYPE_CODES[np.dtype(np.float64)], rows, n_cols, rows * (nnz_r or 1), k, nnz_r or 1))
    chunks = args.chunks if args.chunks else (1 if world == 1 or tiled_shape else 4)
    cr, pieces = partition_rows_cyclic(rows, world, chunks)
    mine = pieces[rank]
    my_rows = sum(n for _, n in mine)

    t0 = time.perf_counter()
    blks = [DeviceCsrBlock.generate(SEED_A, r0, n, n_cols, kind, ra, rb, _lib.VAL_UNIFORM, np.float64, device=dev)
            for r0, n in mine]
    my_nnz = sum(b.nnz for b in blks)
    nnz_total = my_nnz
    if world > 1:
        t = torch.tensor([my_nnz], dtype=torch.int64, device=dev)
        dist.all_reduce(t)
        nnz_total = int(t.item())
    x = gen_dense(SEED_X, 0, n_cols, k, device=dev)
    y_local = torch.empty((chunks, cr, k), dtype=torch.float64, device=dev)
    nnz_local = torch.zeros((chunks, cr), dtype=torch.int32, device=dev)
    if world > 1:
        y_full = torch.empty((chunks * world * cr, k), dtype=torch.float64, device=dev)
        nnz_full = torch.zeros(chunks * world * cr, dtype=torch.int32, device=dev)
    else:
        y_full, nnz_full = y_local.view(chunks * cr, k), nnz_local.view(chunks * cr)
    comp = Compactor(rows, k, np.float64, device=dev)
    torch.cuda.synchronize()
    log(f"rank {rank}: {my_rows:,} rows in {chunks} round(s) of {cr:,}, nnz {my_nnz:,} generated in "
        f"{time.perf_counter() - t0:.1f} s")
    # the SpMM schedule's per-matrix preparation, built once per matrix like
    # the matrix itself (outside the timed region; its cost is reported as
    # plan_ms): the row-block x column-panel copy, or the column-panel plan
    t0 = time.perf_counter()
    panel_cols, tiled, tiled_info = 0, False, None
    if args.schedule != "panel" and k in (1, 32):
        plans = [b.plan_tiled(k, force=args.schedule == "tiled") for b in blks]
        tiled = all(p is not None for p in plans)
        if tiled:
            infos = [p.info() for p in plans]
            tiled_info = {"bytes": sum(i["bytes"] for i in infos), "slots": sum(i["slots"] for i in infos),
                          "panel_cols": infos[0]["panel_cols"]}
        else:
            for b in blks:
                b.tiled = None
    if not tiled:
        for b in blks:
            panel_cols = b.plan(k, args.panel_cols)
    torch.cuda.synchronize()
    plan_ms = (time.perf_counter() - t0) * 1e3
    n_passes = -(-n_cols // panel_cols) if panel_cols else 1
    if tiled:
        log(f"rank {rank}: row-block x column-panel copy {tiled_info}, built in {plan_ms:.1f} ms")
    else:
        log(f"rank {rank}: panel width {panel_cols} ({n_passes} passes), plan {plan_ms:.1f} ms")

    # one set of events per timed step, read after the timed region: no host
    # synchronisation between steps (small configs would time the bubble)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(4)] for _ in range(args.steps)]
    kern_ms, comm_ms, comp_ms = [], [], []
    round_rows = world * cr

    def step(timed):
        if timed:
            ev_k0, ev_k1, ev_c0, ev_c1 = evs[timed - 1]
            ev_k0.record()
        works = []
        for c, b in enumerate(blks):
            b.spmm(x, y_local[c, :b.rows], nnz_local[c, :b.rows])
            if world > 1:  # RCCL all-gather of this round's Y rows (+ nnz counts), overlapped with the next
                works.append(dist.all_gather_into_tensor(y_full[c * round_rows:(c + 1) * round_rows], y_local[c],
                                                         async_op=True))
                works.append(dist.all_gather_into_tensor(nnz_full[c * round_rows:(c + 1) * round_rows],
                                                         nnz_local[c], async_op=True))
        if timed:
            ev_k1.record()
        for w in works:
            w.wait()
        if timed:
            ev_c0.record()
        comp(y_full[:rows], nnz_full[:rows])
        if timed:
            ev_c1.record()

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for i in range(args.steps):
        step(i + 1)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    for ev_k0, ev_k1, ev_c0, ev_c1 in evs:
        kern_ms.append(ev_k0.elapsed_time(ev_k1))
        comm_ms.append(ev_k1.elapsed_time(ev_c0))
        comp_ms.append(ev_c0.elapsed_time(ev_c1))
    log(f"rank {rank}: SpMM kernel ms per timed step: {[round(t, 2) for t in kern_ms]}")
    if world > 1:
        t = torch.tensor([elapsed, float(np.mean(kern_ms))], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kmax = float(t[0]), float(t[1])
    else:
        kmax = float(np.mean(kern_ms))

    verified = None
    if args.verify:
        if rank == 0:  # the whole product on one GPU, compared with the assembled one
            full = DeviceCsrBlock.generate(SEED_A, 0, rows, n_cols, kind, ra, rb, _lib.VAL_UNIFORM, np.float64,
                                           device=dev)
            full.plan(k, args.panel_cols)  # the other schedule than the tiled ranks use: same bits
            y_ref = torch.empty((rows, k), dtype=torch.float64, device=dev)
            nnz_ref = torch.empty(rows, dtype=torch.int32, device=dev)
            full.spmm(x, y_ref, nnz_ref)
            verified = bool(torch.equal(y_ref.view(torch.int64), y_full[:rows].reshape(rows, k).view(torch.int64))
                            and torch.equal(nnz_ref, nnz_full[:rows]))
            del full, y_ref, nnz_ref
            log(f"verify: assembled Y {'==' if verified else '!='} single-GPU Y")
        if world > 1:
            dist.barrier()
    out_nnz = comp.nnz()
    e2e = None
    if world == 1 and not args.no_e2e:
        e2e = end_to_end(args.config, blks, x, comp, step, rows, k)
        log(f"end to end: {e2e}")
    ms_per_step = elapsed / args.steps * 1e3
    value = b_alg(rows, n_cols, nnz_total, k) / (elapsed / args.steps) / 1e9
    # roofline of the dominant kernel (the SpMM: n_passes launches of the
    # panelled kernel, bracketed together by the HIP events): algorithmic
    # bytes of THIS rank's SpMM over its measured average duration
    b_launch = b_alg(my_rows, n_cols, my_nnz, k)
    achieved = b_launch / (float(np.mean(kern_ms)) / 1e3) / 1e9
    achieved_gather = b_gather(my_rows, my_nnz, k) / (float(np.mean(kern_ms)) / 1e3) / 1e9
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1:
            log("timing cpu baseline ...")
            cpu = cpu_baseline(args.config, args.cpu_sample_rows)
        traffic, traffic_src = args.traffic_bytes, "--traffic-bytes" if args.traffic_bytes else None
        pmc_json = os.path.join(ROOT, "profiles", f"pmc_traffic_{args.config}.json")
        if traffic is None and world == 1 and os.path.exists(pmc_json):
            # rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this kernel on
            # this config (separate runs), corrected per MI355X_MICROARCH.md
            with open(pmc_json) as f:
                pmc = json.load(f)
            if pmc.get("panel_cols", 0) == panel_cols and pmc.get("schedule", "panel") == (
                    "tiled" if tiled else "panel"):  # same schedule as this run
                traffic = pmc["traffic_bytes_per_launch"] * pmc.get("launches_per_spmm", 1)
                traffic_src = os.path.relpath(pmc_json, ROOT)
        line = {
            "metric": "CSR x dense SpMM effective GB/s (B_alg / step time); nnz/s",
            "value": round(value, 2),
            "unit": "GB/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": round(ms_per_step, 3),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (SplitMix64 random CSR, sorted distinct uniform columns, values U[0.5,1.5); "
                    "generated on device from seeds 1000/1001)",
            "config": {
                "workload": f"{args.config}: {rows:,} x {n_cols:,} CSR, "
                            + (f"{nnz_r} nnz/row" if nnz_r else f"Binomial({n_cols}, {C1_P:g}) nnz/row")
                            + f" ({100.0 * nnz_total / rows / n_cols:.3g} % density, nnz {nnz_total:,}) x {k}-column dense RHS, "
                            f"f64; step = SpMM + {'RCCL all-gather of Y + ' if world > 1 else ''}compaction "
                            f"to Csr",
                "rows": rows, "n_cols": n_cols, "nnz": nnz_total, "rhs_cols": k,
                "parallelism": f"row-block x{world}" + (f" (block-cyclic, {chunks} rounds) + overlapped all-gather"
                                                         if world > 1 else ""),
                "schedule": f"row-block x column-panel copy (spmm_tiled_k{k})" if tiled else
                            ("column panels" if panel_cols else "one pass"),
                "panel_cols": tiled_info["panel_cols"] if tiled else panel_cols, "passes": n_passes,
                "plan_ms": round(plan_ms, 1),
                "tiled_copy": tiled_info,
            },
            "nnz_per_s": round(nnz_total / (elapsed / args.steps), 1),
            "hbm_frac_of_peak": round(value / (world * HBM_PEAK_GBS), 5),
            "breakdown_ms": {
                "spmm_kernel_mean": round(float(np.mean(kern_ms)), 3),
                "spmm_kernel_max_over_ranks": round(kmax, 3),
                "allgather_mean": round(float(np.mean(comm_ms)), 3),
                "compaction_mean": round(float(np.mean(comp_ms)), 3),
            },
            "output_nnz": out_nnz,
            "verified_vs_single_gpu": verified,
            "roofline": {
                "bound": "hbm",
                "kernel": kernel_label(my_rows, my_nnz, k, panel_cols, tiled),
                "model": "B_alg (SURVEY.md §8d canonical: X and Y counted once)",
                "launches_per_spmm": n_passes,
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "traffic_GBps": round(traffic / (float(np.mean(kern_ms)) / 1e3) / 1e9, 1) if traffic else None,
                "bytes_per_launch_alg": b_launch,
            },
            "roofline_gather": {
                "bound": "hbm",
                "model": "B_gather (SURVEY.md §8d traffic model: every nnz gathers its whole X row)",
                "achieved": round(achieved_gather, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved_gather / HBM_PEAK_GBS, 5),
                "bytes_per_launch_gather": b_gather(my_rows, my_nnz, k),
            },
            "end_to_end_ms": e2e,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
