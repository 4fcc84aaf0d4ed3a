#!/usr/bin/env python3
"""bench.py -- CSR x dense SpMM throughput on MI355X (BASELINE.json metric:
"CSR x dense SpMM effective GB/s (% HBM3E peak) at 1/2/4/8 GPUs; nnz/s").

Workload (BASELINE.json north_star target / configs[3]): A = 10M x 10M
synthetic random CSR, 1000 nnz per row (0.01 % density, nnz = 1e10), f64,
times a dense 10M x 32 f64 RHS. It fits one MI355X (A 120 GB + X/Y 5 GB of
288 GB HBM), so N=1 runs the whole matrix on one GPU.

The measured path is the library's multi-GPU C-ABI (include/bsm.h
"multi-GPU", csrc/multi.hip), the same entry points a Rust `mul_dense`
binds: one process per GPU, each rank's context made by
bsm_multi_create_rank from an RCCL id that rank 0 ships through
torch.distributed (backend nccl = RCCL), or, run without a launcher, by
bsm_multi_create(1) (ncclCommInitAll over the one GPU). The CSR is cut into
`--chunks` x N nnz-balanced row blocks (block c*N + g on rank g, computed in
round c), generated on each rank's device. X is generated on rank 0 and
replicated by the library's ncclBroadcast (untimed setup). Every round's Y
blocks are all-gathered in place by the library's own RCCL communicator on a
communication stream, overlapping the next round's SpMM, and every rank
compacts the assembled Y into the output Csr. Total work is fixed as N grows
("strong").

One step = the hot path of Csr::mul_dense (src/sparse.rs:426-446) over the
whole matrix: SpMM rounds -> RCCL all-gathers of Y and of the per-row
nonzero counts -> compaction of Y into the output Csr (zero-dropping insert,
sparse.rs:229). Inputs are resident in HBM before timing starts.

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
# The L2-served gather ceiling of the tiled kernel's own inner loop (same
# pipeline, 16-B/lane gathers, LDS read-add-write per chunk) on a static X
# table that stays in each XCD's L2: scripts/perf/gather_ceiling.sh,
# profiles/r03_gather_ceiling.log ("static 2 MiB table, LDS update" line).
# It is the peak of roofline_gather: the C4 gathers (2.56 TB) cannot be served
# faster than the L2 serves them.
L2_GATHER_PEAK_GBS = 17_030.0  # 17.03 TB/s: "mode 2 ... 8191" line (0.987 ms for 6.57e7 entries)
L2_GATHER_PEAK_SRC = "profiles/r03_gather_ceiling.log"
# The Infinity-Cache service rate of L2 misses. Every byte a kernel misses
# in L2 (its PMC traffic: X rows it gathers past L2, the index/value stream,
# the writes) is served by the Infinity Cache or HBM. The ceiling is the
# fastest Infinity-Cache-served gather rate measured on this chip:
# MI355X_MICROARCH.md §Indexed rows, 38 MB table of uniformly random rows,
# 8.6 TB/s. Our own probe (the tiled loop at C4 with one panel and every
# column folded into a 256 MB table: BSM_TILED_PSHIFT=24,
# BSM_TILED_PROBE_MASK=2^20-1) moved 2.68 TB of L2-miss bytes (2.56 TB of
# gathers + the 124 GB stream) in 358 ms: 7.50 TB/s (a 1 GB table: the same);
# roofline_gather reports the kernel's fraction of that too.
IC_SERVICE_PEAK_GBS = 8_600.0
IC_SERVICE_PEAK_SRC = "MI355X_MICROARCH.md §Indexed rows (38 MB table, Infinity Cache)"
IC_PROBE_GBS = 7_500.0
IC_PROBE_SRC = "profiles/r04_b_c4_ic_gather_probe.log"
# k = 1 (C2, spmm_tiled_k1): the same kernel with every gather confined to one
# L2-resident 2 MiB panel (BSM_TILED_K1_PROBE=262143): 59 us at C2, i.e. C2's
# B_gather (216,000,008 B) at 3,661 GB/s. Each 8-B gather moves a 128-B line
# into L1 that no other gather of the CU re-uses.
K1_GATHER_PEAK_GBS = 3_661.0
K1_GATHER_PEAK_SRC = "profiles/r02_f_c2_gather_probe.log"
ROWLEN_CONST, ROWLEN_BINOMIAL = 0, 2  # bsm_synth.h row-length families
SEED_A, SEED_X = 1000, 1001


def b_alg(rows, n_cols, nnz, k, es=8):
    """SURVEY.md §8d canonical bytes (es = value size: 8 for f64, 4 for f32):
    8(N+1) + (4 + es) nnz + es n_cols k + es N k."""
    return 8 * (rows + 1) + (4 + es) * nnz + es * n_cols * k + es * rows * k


def b_gather(rows, nnz, k, es=8):
    """SURVEY.md §8d traffic model: every nnz gathers its whole X row (no reuse
    beyond the caches): 8(N+1) + (4 + es) nnz + es nnz k + es N k."""
    return 8 * (rows + 1) + (4 + es) * nnz + es * nnz * k + es * rows * k


def gather_ceiling(tiled, k, x_bytes, gather_bytes, traffic):
    """The gather ceiling that bounds this schedule (measured, per config).
    The tiled k = 1 copy (C2) moves a 128-B line per 8-B gather: its own
    one-panel probe. Otherwise a gather is served by L2 or, when it misses,
    by the Infinity Cache; hits and misses overlap, so the kernel cannot be
    faster than either side alone: peak = min(L2 gather ceiling, IC service
    ceiling x B_gather / miss bytes), B_gather and the miss bytes (the
    kernel's PMC traffic, profiles/pmc_traffic_<config>.json) per SpMM. Without a PMC
    record: the L2 ceiling for the tiled copy, the IC ceiling for a row
    kernel on an X beyond L2."""
    if tiled and k == 1:
        return {"bound": "l2_line_gather_k1", "peak": K1_GATHER_PEAK_GBS, "peak_source": K1_GATHER_PEAK_SRC,
                "peak_model": "the same kernel, every gather in one L2-resident 2 MiB panel (BSM_TILED_K1_PROBE)"}
    l2 = {"bound": "l2_gather", "peak": L2_GATHER_PEAK_GBS, "peak_source": L2_GATHER_PEAK_SRC,
          "peak_model": "the same inner loop on a static L2-resident X table"}
    if traffic:
        ic = IC_SERVICE_PEAK_GBS * gather_bytes / traffic
        out = l2 if L2_GATHER_PEAK_GBS <= ic else {
            "bound": "ic_miss_service", "peak": round(ic, 1),
            "peak_source": f"{IC_SERVICE_PEAK_SRC}; miss bytes: PMC traffic",
            "peak_model": "IC service ceiling x B_gather / the kernel's L2-miss bytes"}
        return dict(out, peak_rule="min(L2 gather ceiling, IC service ceiling x B_gather / miss bytes)",
                    ic_service_peak=IC_SERVICE_PEAK_GBS, miss_bytes_per_spmm=traffic,
                    ic_probe_peak=round(IC_PROBE_GBS * gather_bytes / traffic, 1), ic_probe_source=IC_PROBE_SRC)
    if not tiled and x_bytes > (32 << 20):
        return {"bound": "ic_gather", "peak": IC_SERVICE_PEAK_GBS, "peak_source": IC_SERVICE_PEAK_SRC,
                "peak_model": "uniformly random row gathers served by the Infinity Cache (no L2 re-use, no PMC "
                              "record for this run)"}
    return l2


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


def end_to_end(cfg_name, m, x, dev, iters=3):
    """What a caller of the public API pays (host buffers in and out, A
    resident on the device as the mirrors cache it), next to the
    device-resident step:
      multi_api_ms = bsm_mcsr_mul_dense (host X columns uploaded to every
        device, the step, the output Csr as a handle) + bsm_csr_download into
        usize/T host arrays: the multi-GPU path a Rust mul_dense takes;
      public_api_ms (host-sized configs) = Csr.mul_dense(Dense) of the Python
        mirror on one GPU (bsm_csr_mul_dense + download), host Dense in, host
        Csr out."""
    from basic_sparse_matrix_amd import Csr, Dense
    from basic_sparse_matrix_amd.device import DeviceCsrBlock

    out = {}
    rows, n_cols, k = m.rows, m.cols, int(x.shape[1])
    xh = x.cpu().numpy()
    x_cols = [np.ascontiguousarray(xh[:, j]) for j in range(k)]
    ts, n_out = [], 0
    for _ in range(iters):
        t0 = time.perf_counter()
        dc = m.mul_dense_cols(x_cols, n_cols)
        rp, ci, v = dc.download()
        ts.append(time.perf_counter() - t0)
        n_out = int(rp[-1])
        del dc, rp, ci, v
    out["multi_api_ms"] = round(float(np.median(ts)) * 1e3, 3)
    out["h2d_bytes"] = int(n_cols * k * 8)
    out["d2h_bytes"] = int((rows + 1) * 8 + n_out * 16)
    if m.nnz <= 200_000_000:
        kind, ra, rb = rowlen_spec(cfg_name)
        b = DeviceCsrBlock.generate(SEED_A, 0, rows, n_cols, kind, ra, rb, 0, np.float64, device=dev)
        a = Csr.from_csr_arrays((rows, n_cols), b.row_ptr.cpu().numpy().astype(np.uint64),
                                b.col.cpu().numpy().astype(np.uint64), b.vals.cpu().numpy())
        del b
        xd = Dense.from_columns(x_cols)
        a.mul_dense(xd)  # first call uploads and caches A on the device (untimed, like the bench's setup)
        ts = []
        for _ in range(max(iters, 20 if cfg_name in ("c1", "c2", "c3") else iters)):
            t0 = time.perf_counter()
            a.mul_dense(xd)
            ts.append(time.perf_counter() - t0)
        out["public_api_ms"] = round(float(np.median(ts)) * 1e3, 4)
        out["public_api_calls"] = len(ts)
        # the same call split: time inside the C-ABI (bsm_csr_mul_dense: X
        # upload + SpMM + compaction; bsm_csr_download into fresh usize / f64
        # arrays) and the caller freeing the previous result (its host pages)
        import ctypes

        lib = _lib_load()
        dev_a = a._device()
        ptrs = _ptr_array(x_cols)
        lib_ts, free_ts, prev = [], [], None
        for _ in range(len(ts)):
            t0 = time.perf_counter()
            h = ctypes.c_void_p()
            _check(lib.bsm_csr_mul_dense(dev_a.handle, k, n_cols, ptrs, ctypes.byref(h)))
            dc = _DeviceCsr(h.value)
            res = dc.download()
            t1 = time.perf_counter()
            prev, old = res, prev
            del old
            t2 = time.perf_counter()
            lib_ts.append(t1 - t0)
            free_ts.append(t2 - t1)
            del dc
        out["public_api_split_ms"] = {"in_library": round(float(np.median(lib_ts)) * 1e3, 4),
                                      "caller_frees_previous_result": round(float(np.median(free_ts)) * 1e3, 4)}
        del prev, res
        # the same public call with the host result pool off: fresh numpy
        # arrays per result, faulted in and later unmapped (hostpool.py)
        os.environ["BSM_HOST_POOL"] = "0"
        try:
            ts = []
            for _ in range(10):
                t0 = time.perf_counter()
                a.mul_dense(xd)
                ts.append(time.perf_counter() - t0)
            out["public_api_fresh_arrays_ms"] = round(float(np.median(ts)) * 1e3, 4)
        finally:
            os.environ.pop("BSM_HOST_POOL", None)
    return out


def _lib_load():
    from basic_sparse_matrix_amd import _lib

    return _lib.load()


def _ptr_array(arrs):
    from basic_sparse_matrix_amd import _lib

    return _lib.ptr_array(arrs)


def _check(rc):
    from basic_sparse_matrix_amd import _lib

    _lib.check(rc)


def _DeviceCsr(h):
    from basic_sparse_matrix_amd import _lib

    return _lib.DeviceCsr(h)


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
            for _ in range(7 if name != "ss_mul" else (3 if e <= 100_000 else 1)):  # median: host noise
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


def verify_rows(m, x, k, dev, kind, ra, rb, full):
    """Rank 0: compare the assembled Y and row counts with a single-GPU
    recomputation by the other schedule (column panels / one pass), bit for
    bit. `full`: the whole matrix (needs a second copy of A); else blocks of
    2048 rows around every piece bound plus the first and last rows (the
    assembly's seams), so C4 fits beside its copy."""
    from basic_sparse_matrix_amd.device import DeviceCsrBlock

    rows, n_cols = m.rows, m.cols
    y_all = torch.empty((rows, k), dtype=torch.float64, device=dev)
    nnz_all = torch.empty(rows, dtype=torch.int32, device=dev)
    m.copy_y(0, y_all.data_ptr(), nnz_all.data_ptr())
    if full:
        spans = [(0, rows)]
    else:
        pts = sorted(set(int(b) for b in m.bounds()) | {0, rows})
        spans, last = [], -1
        for p in pts:
            a, b = max(0, p - 1024), min(rows, p + 1024)
            if a < last:
                a = last
            if b > a:
                spans.append((a, b))
                last = b
    checked = 0
    for a, b in spans:
        blk = DeviceCsrBlock.generate(SEED_A, a, b - a, n_cols, kind, ra, rb, 0, np.float64, device=dev)
        blk.plan(k)
        y_ref = torch.empty((b - a, k), dtype=torch.float64, device=dev)
        nnz_ref = torch.empty(b - a, dtype=torch.int32, device=dev)
        blk.spmm(x, y_ref, nnz_ref)
        ok = torch.equal(y_ref.view(torch.int64), y_all[a:b].view(torch.int64)) and torch.equal(nnz_ref, nnz_all[a:b])
        del blk, y_ref, nnz_ref
        if not ok:
            log(f"verify: rows [{a}, {b}) differ")
            return False, checked
        checked += b - a
    return True, checked


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=5)
    ap.add_argument("--warmup", type=int, default=2)
    ap.add_argument("--config", default="c4", choices=sorted(CONFIGS))
    ap.add_argument("--dtype", default="f64", choices=("f64", "f32"),
                    help="value type of A, X and Y (BASELINE's configs are f64; f32 = the generic-T path)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-rows", type=int, default=100_000,
                    help="rows of the CPU baseline sample (configs with more rows are extrapolated)")
    ap.add_argument("--panel-cols", type=int, default=None,
                    help="column-panel width of the SpMM schedule (default: the library's choice; 0 = one pass)")
    ap.add_argument("--schedule", default="auto", choices=("auto", "tiled", "panel"),
                    help="SpMM schedule: auto = the library's choice (row-block x column-panel copy when "
                         "wanted, else column panels), tiled = the copy whenever possible, panel = never the copy")
    ap.add_argument("--chunks", type=int, default=0,
                    help="rounds of the row partition (pieces = chunks x N; 0: 1 at N=1 or with the tiled copy, "
                         "4 otherwise)")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend under a launcher (nccl = RCCL)")
    ap.add_argument("--exchange", default="rccl", choices=("rccl", "gloo"),
                    help="how the ranks' Y slots are assembled: rccl = the library's in-place all-gathers; gloo = "
                         "external rank contexts (bsm_multi_create_external) and distributed.exchange_slots over "
                         "the launcher's group on the host (several ranks on one GPU: a logic check of the N > 1 "
                         "path, not a measurement)")
    ap.add_argument("--verify", action="store_true",
                    help="rank 0 recomputes Y on its own GPU by another schedule and checks the assembled Y bit for "
                         "bit (whole matrix up to 2e9 nnz, else the rows around every piece bound)")
    ap.add_argument("--traffic-bytes", type=float, default=None,
                    help="PMC-measured HBM bytes per SpMM launch (from profiles/), reported as roofline.traffic")
    ap.add_argument("--no-e2e", action="store_true", help="skip the end-to-end (host buffers in/out) figures")
    ap.add_argument("--ref-benches", default=None,
                    help="comma list of the reference's own criterion benches to run instead "
                         "(sd_mul,ss_add,ss_mul; one JSON line per size)")
    args = ap.parse_args()
    if args.panel_cols is not None:
        os.environ["BSM_SPMM_PANEL_COLS"] = str(args.panel_cols)
    if args.ref_benches:
        ref_bench_suite(which=tuple(args.ref_benches.split(",")))
        return

    launched = "WORLD_SIZE" in os.environ  # torch.distributed.run sets it, also at N = 1
    external = args.exchange == "gloo"
    if external and not launched:
        ap.error("--exchange gloo needs a launcher (torch.distributed.run)")
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        log(f"WORLD_SIZE={world} but --gpus={args.gpus}; using WORLD_SIZE")
    ordinal = local_rank % max(1, torch.cuda.device_count())
    torch.cuda.set_device(ordinal)
    dev = torch.device("cuda", ordinal)
    backend = None
    if launched:
        backend = "gloo" if external else args.backend
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=dev)
        else:
            dist.init_process_group(backend)

    from basic_sparse_matrix_amd import _lib
    from basic_sparse_matrix_amd.device import gen_dense
    from basic_sparse_matrix_amd.multi import MultiCsr, MultiGpu, unique_id

    rows, n_cols, nnz_r, k = CONFIGS[args.config]
    kind, ra, rb = rowlen_spec(args.config)
    f32 = args.dtype == "f32"
    np_dt, torch_dt, es = (np.float32, torch.float32, 4) if f32 else (np.float64, torch.float64, 8)
    if f32 and args.verify:
        ap.error("--verify compares f64 Y; the f32 path is checked by tests/test_gpu_tiled.py")
    lib0 = _lib.load()
    tiled_shape = args.schedule != "panel" and k in (1, 32) and bool(lib0.bsm_dev_tiled_wanted(
        _lib.DTYPE_CODES[np.dtype(np_dt)], rows, n_cols, rows * (nnz_r or 1), k, nnz_r or 1))
    # the tiled copy's persistent grid wants every CU, so by default its rank
    # runs one round and the all-gather follows it (--chunks overrides)
    chunks = args.chunks if args.chunks else (1 if world == 1 or tiled_shape else 4)

    # the library's RCCL context: the id travels over torch.distributed
    t0 = time.perf_counter()
    if external:
        ctx = MultiGpu.external(world, rank, ordinal)
    elif launched:
        obj = [unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0)
        ctx = MultiGpu.for_rank(obj[0], world, rank, ordinal)
    else:
        ctx = MultiGpu(1, devices=[ordinal])
    comm_init_ms = (time.perf_counter() - t0) * 1e3

    t0 = time.perf_counter()
    m = MultiCsr.generate(ctx, SEED_A, rows, n_cols, kind, ra, rb, _lib.VAL_UNIFORM, np_dt, chunks=chunks)
    gen_ms = (time.perf_counter() - t0) * 1e3
    nnz_total = m.nnz
    bounds = m.bounds()
    my_pieces = [(int(bounds[c * world + rank]), int(bounds[c * world + rank + 1])) for c in range(chunks)]
    my_rows = sum(b - a for a, b in my_pieces)
    # the rows' nnz (the generator's row lengths): constant-length configs by count
    my_nnz = my_rows * nnz_r if nnz_r else None
    x = torch.empty((n_cols, k), dtype=torch_dt, device=dev)
    if rank == 0 or external:  # external ranks have no communicator: each makes the replica itself
        x.copy_(gen_dense(SEED_X, 0, n_cols, k, dtype=np_dt, device=dev))
    torch.cuda.synchronize()
    if not external:
        ctx.broadcast([x.data_ptr()], x.numel() * es, root=0)  # X replicated over RCCL (untimed setup)
    log(f"rank {rank}: pieces {my_pieces} of {m.pieces} ({chunks} round(s)), nnz {nnz_total:,} in total, generated in "
        f"{gen_ms:.0f} ms; RCCL context {comm_init_ms:.0f} ms")
    # the output Csr is returned on rank 0 (Csr::mul_dense has one caller):
    # the other ranks keep the gathered Y only, no output buffers, no compaction
    if world > 1:
        m.set_output_rank(0)
    # the schedule's per-matrix preparation (outside the timed region, like the
    # matrix itself; reported per phase as plan_ms)
    plan = m.prepare(k, args.schedule)
    pinfo = m.plan_info()
    tiled = pinfo["tiled_pieces"] == pinfo["local_pieces"] and pinfo["tiled_pieces"] > 0
    panel_cols = 0 if tiled else pinfo["panel_cols"]
    n_passes = -(-n_cols // panel_cols) if panel_cols else 1
    log(f"rank {rank}: schedule {pinfo}, plan {plan}")
    if my_nnz is None:  # variable row lengths (C1): count them on the device
        from basic_sparse_matrix_amd.device import DeviceCsrBlock

        my_nnz = sum(DeviceCsrBlock.generate(SEED_A, a, b - a, n_cols, kind, ra, rb, 0, np.float64, device=dev).nnz
                     for a, b in my_pieces)

    xp = [x.data_ptr()]

    def step():
        m.step(xp)
        if external:  # the slots over the host group, then the compaction
            from basic_sparse_matrix_amd.distributed import exchange_slots

            m.sync()
            exchange_slots(m, world, rank, chunks)
            m.compact()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    m.reset_times()
    if launched:
        dist.barrier()
    torch.cuda.synchronize()
    t_start = time.perf_counter()
    for _ in range(args.steps):
        step()
    torch.cuda.synchronize()
    if launched:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t_start
    times = m.step_times(0)[:args.steps]
    kern_ms = [t["spmm"] for t in times]
    comm_ms = [t["allgather_tail"] for t in times]
    comp_ms = [t["compaction"] for t in times]
    log(f"rank {rank}: SpMM ms per timed step: {[round(t, 2) for t in kern_ms]}")
    if launched:
        t = torch.tensor([elapsed, float(np.mean(kern_ms))], dtype=torch.float64,
                         device=dev if backend == "nccl" else "cpu")
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kmax = float(t[0]), float(t[1])
    else:
        kmax = float(np.mean(kern_ms))

    verified, verified_rows = None, 0
    if args.verify:
        if rank == 0:
            verified, verified_rows = verify_rows(m, x, k, dev, kind, ra, rb, full=nnz_total <= 2_000_000_000)
            log(f"verify: assembled Y {'==' if verified else '!='} single-GPU Y on {verified_rows:,} rows")
        if launched:
            dist.barrier()
    e2e = None
    if world == 1 and not args.no_e2e and not f32:
        e2e = end_to_end(args.config, m, x, dev)
        log(f"end to end: {e2e}")
    ms_per_step = elapsed / args.steps * 1e3
    value = b_alg(rows, n_cols, nnz_total, k, es) / (elapsed / args.steps) / 1e9
    # roofline of the dominant kernel (the SpMM rounds on the compute stream,
    # bracketed by the library's HIP events): algorithmic bytes of THIS rank's
    # SpMM over its measured average duration
    b_launch = b_alg(my_rows, n_cols, my_nnz, k, es)
    t_k = float(np.mean(kern_ms)) / 1e3
    achieved = b_launch / t_k / 1e9
    achieved_gather = b_gather(my_rows, my_nnz, k, es) / t_k / 1e9
    if rank == 0:
        cpu = None
        if not args.no_cpu_baseline and world == 1 and not f32:
            log("timing cpu baseline ...")
            cpu = cpu_baseline(args.config, args.cpu_sample_rows)
        traffic, traffic_src, pmc = args.traffic_bytes, "--traffic-bytes" if args.traffic_bytes else None, None
        pmc_json = os.path.join(ROOT, "profiles", f"pmc_traffic_{args.config}.json")
        if traffic is None and world == 1 and chunks == 1 and os.path.exists(pmc_json):
            # rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes of this kernel on
            # this config (separate runs), corrected per MI355X_MICROARCH.md
            with open(pmc_json) as f:
                pmc = json.load(f)
            if pmc.get("panel_cols", 0) == panel_cols and pmc.get("schedule", "panel") == (
                    "tiled" if tiled else "panel") and not f32:  # same schedule and dtype as this run
                traffic = pmc["traffic_bytes_per_launch"] * pmc.get("launches_per_spmm", 1)
                traffic_src = os.path.relpath(pmc_json, ROOT)
            else:
                pmc = None
        gceil = gather_ceiling(tiled, k, n_cols * k * es, b_gather(my_rows, my_nnz, k, es), traffic)
        solo_rccl = os.environ.get("BSM_MULTI_SOLO_RCCL") == "1"
        comm = ((f"external rank contexts, Y slots exchanged over torch.distributed {backend} on the host "
                 f"({world} ranks; a logic check, not a measurement)") if external else
                ("one rank: no collective (the library skips the all-gathers, which have nothing to move at one "
                 "rank; BSM_MULTI_SOLO_RCCL=1 runs them)" + (f"; context id over torch.distributed {backend}"
                                                             if launched else ""))
                if world == 1 and not solo_rccl else
                (f"library RCCL all-gather (bsm_mcsr_step; {world} rank(s)"
                 + (f", context id over torch.distributed {backend})" if launched else ", ncclCommInitAll)")))
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
            "dtype": args.dtype,
            "data": "synthetic (SplitMix64 random CSR, sorted distinct uniform columns, values U[0.5,1.5); "
                    "generated on device from seeds 1000/1001)",
            "config": {
                "workload": f"{args.config}: {rows:,} x {n_cols:,} CSR, "
                            + (f"{nnz_r} nnz/row" if nnz_r else f"Binomial({n_cols}, {C1_P:g}) nnz/row")
                            + f" ({100.0 * nnz_total / rows / n_cols:.3g} % density, nnz {nnz_total:,}) x {k}-column "
                              f"dense RHS, {args.dtype}; step = SpMM rounds + RCCL all-gather of Y + compaction to Csr",
                "rows": rows, "n_cols": n_cols, "nnz": nnz_total, "rhs_cols": k,
                "parallelism": f"row-block x{world}, {chunks} round(s) of {world} nnz-balanced pieces",
                "comm": comm,
                "schedule": f"row-block x column-panel copy (spmm_tiled_k{k}; Y rows in LDS)" if tiled else
                            ("column panels" if panel_cols else
                             "one pass, row per wave" + (" (spmm_k32_f64_rows4, 4 rows per wave): no LDS X panel, "
                                                          "since at 10 nnz/row an X row meets ~0.2 other entries per "
                                                          "L2 lifetime; the LDS row-block copy measured 0.63 ms "
                                                          "against 0.42 (profiles/r04_b_c3_rows4_vs_tiled.log)"
                                                          if k == 32 and nnz_total <= 24 * rows else "")),
                "panel_cols": pinfo["panel_cols"], "passes": n_passes,
                "plan_ms": plan,
                "generate_ms": round(gen_ms, 1),
                "comm_init_ms": round(comm_init_ms, 1),
                "tiled_copy_bytes": pinfo["copy_bytes"] if tiled else None,
            },
            "nnz_per_s": round(nnz_total / (elapsed / args.steps), 1),
            "hbm_frac_of_peak": round(value / (world * HBM_PEAK_GBS), 5),
            "breakdown_ms": {
                "spmm_kernel_mean": round(float(np.mean(kern_ms)), 3),
                "spmm_kernel_max_over_ranks": round(kmax, 3),
                "allgather_tail_mean": round(float(np.mean(comm_ms)), 3),
                "compaction_mean": round(float(np.mean(comp_ms)), 3),
                "spmm_kernel_per_step": [round(t, 3) for t in kern_ms],
            },
            "verified_vs_single_gpu": verified,
            "verified_rows": verified_rows if args.verify else None,
            "roofline": {
                "bound": "hbm",
                "kernel": kernel_label(my_rows, my_nnz, k, panel_cols, tiled),
                "model": "B_alg (SURVEY.md §8d canonical: X and Y counted once)",
                "launches_per_spmm": n_passes * chunks,
                "achieved": round(achieved, 2),
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 5),
                "traffic": traffic,
                "traffic_source": traffic_src,
                "traffic_GBps": round(traffic / t_k / 1e9, 1) if traffic else None,
                "traffic_split": {key: pmc[key] for key in ("stream_bytes", "gather_bytes", "write_bytes")
                                  if key in pmc} if pmc else None,
                "bytes_per_launch_alg": b_launch,
            },
            "roofline_gather": dict(
                gceil,
                model="B_gather (SURVEY.md §8d traffic model: every nnz gathers its whole X row)",
                achieved=round(achieved_gather, 2),
                unit="GB/s",
                frac=round(achieved_gather / gceil["peak"], 5),
                **({"ic_probe_frac": round(achieved_gather / gceil["ic_probe_peak"], 5)}
                   if "ic_probe_peak" in gceil else {}),
                bytes_per_launch_gather=b_gather(my_rows, my_nnz, k, es),
            ),
            "end_to_end_ms": e2e,
            "cpu_baseline": cpu,
        }
        print(json.dumps(line), flush=True)
    del m
    ctx.close()
    if launched:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
