#!/usr/bin/env python3
"""C5 (north_star config 5): 2D 5-point Poisson on a g x g grid (natural
ordering, N = g^2, band b = g), b = A x_true, solve(A, b) on the GPU through
the reference API (lib.rs:11-24): cholesky_decomp -> transpose -> forward ->
backward substitution. Prints ONE JSON line per order (reference = bit-exact
operation order; blocked = reassociated, within 1e-6 on f64) with

* wall time through the public API (host b in, host x out) and the device
  time of every stage (HIP events on the library's stream, bsm_stage_times);
* the factor's flop roofline (N b^2 flops, the band Cholesky's multiply-add
  pairs x 2, against the 78.6 TF/s f64 peak of MI355X_MICROARCH.md) and each
  triangular solve's byte roofline (the band of L, 8 N (b+1) bytes, read
  once, against 8 TB/s);
* the CPU baseline: the oracle's band restatement of the same solve (the
  reference's order, one thread; the literal O(N^4) reference loops are out
  of reach beyond N ~ 256), timed on this host's cores on the leading 25 grid
  rows of the system and scaled by N/R (per-row work is constant past the
  first g rows), with a whole 250^2 solve beside it;
* the error of x against x_true (and, for the reference order, bit-equality
  with the committed full-size oracle fixture, tests/golden/c5_poisson_1000.json).
"""
import argparse
import hashlib
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from basic_sparse_matrix_amd import Csr, Dense, _lib, solve  # noqa: E402
from oracle import pyoracle as orc  # noqa: E402  (inputs, the CPU baseline and the check only)

F64_PEAK_TFS = 78.6
HBM_PEAK_GBS = 8000.0


def system(g, dt):
    rp, ci, v = orc.poisson2d(g)
    n = g * g
    x_true = orc.gen_x_cols(1002, n, 1)[0]
    rows = np.repeat(np.arange(n), np.diff(rp.astype(np.int64)))
    b = np.zeros(n)
    np.add.at(b, rows, v * x_true[ci.astype(np.int64)])
    return rp, ci, v.astype(dt), b.astype(dt), x_true


def band_kernel():
    """The reference-order factor kernel the library runs."""
    return "band_chol5"


def leading_system(g, rows_g):
    """The leading principal block of the g x g system: the first rows_g grid
    rows (R = rows_g * g unknowns, band g). Its band Cholesky is the first R
    rows of the full factor, and every row past the first g costs the same
    (g^2/2 multiply-add pairs), so its time x N/R is the full solve's."""
    rp, ci, v = orc.poisson2d(g)
    R = rows_g * g
    lo = rp[:R + 1].astype(np.int64)
    keep = ci[:lo[-1]].astype(np.int64) < R
    row_of = np.repeat(np.arange(R), np.diff(lo))
    rp_s = np.concatenate([[0], np.cumsum(np.bincount(row_of[keep], minlength=R))]).astype(np.uint64)
    ci_s, v_s = ci[:lo[-1]][keep], v[:lo[-1]][keep]
    x_true = orc.gen_x_cols(1002, R, 1)[0]
    b = np.zeros(R)
    np.add.at(b, row_of[keep], v_s * x_true[ci_s.astype(np.int64)])
    return R, rp_s, ci_s, v_s, b


def cpu_baseline(fixture, g=1000, sample_rows_g=25, small=250):
    """The oracle's band restatement of solve (the reference's operation order,
    one thread of THIS host: on the GPU box, the node's own cores) on a bounded
    sample: the leading sample_rows_g grid rows of the g x g system (its factor
    is the first rows of the full factor; transpose and the tri-solves are
    linear in rows too), scaled by N/R. A whole small system (small^2) is
    timed beside it. The full 1000^2 run of the build container (the committed
    fixture's cpu_seconds) is kept as a cross-check."""
    n = g * g
    R, rp, ci, v, b = leading_system(g, sample_rows_g)
    t0 = time.perf_counter()
    orc.solve(R, rp, ci, v, [b], band=True)
    t_sample = time.perf_counter() - t0
    est = t_sample * n / R
    rp2, ci2, v2, b2, _ = system(small, np.float64)
    t0 = time.perf_counter()
    orc.solve(small * small, rp2, ci2, v2, [b2], band=True)
    t_small = time.perf_counter() - t0
    container = float(sum(fixture["cpu_seconds"].values())) if fixture and fixture.get("cpu_seconds") else None
    return {
        "value_s": round(est, 2),
        "unit": "s per solve",
        "cores": 1,
        "kind": "port",
        "sample": (f"oracle band restatement of solve (lib.rs:11-24, reference operation order; C, -O2 "
                   f"-ffp-contract=off, 1 thread) timed on this host on the leading {sample_rows_g} grid rows "
                   f"of the {g}^2 system (R = {R:,} of N = {n:,} unknowns, band {g}: {t_sample:.2f} s), "
                   f"x N/R = {n / R:g}"),
        "sample_s": round(t_sample, 3),
        "measured_s": {f"{small}x{small}": round(t_small, 3)},
        "build_container_full_run_s": round(container, 1) if container else None,
        "host_cpus": os.cpu_count(),
    }


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--g", type=int, default=1000)
    ap.add_argument("--dtype", default="f64", choices=("f64", "f32"))
    ap.add_argument("--reps", type=int, default=2, help="timed solves per order (after one warm-up)")
    ap.add_argument("--orders", default="reference,blocked,nd")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample-grid-rows", type=int, default=25,
                    help="CPU baseline: leading grid rows of the system timed on this host (x N/R)")
    args = ap.parse_args()
    dt = np.float64 if args.dtype == "f64" else np.float32
    g = args.g
    n = g * g
    rp, ci, v, b, x_true = system(g, dt)
    A = Csr.from_csr_arrays((n, n), rp, ci, v)
    B = Dense.from_columns([b])
    fixture = None
    fx_path = os.path.join(ROOT, "tests", "golden", f"c5_poisson_{g}.json")
    if os.path.exists(fx_path) and args.dtype == "f64":
        with open(fx_path) as f:
            fixture = json.load(f)
    cpu = None if args.no_cpu_baseline else cpu_baseline(fixture, g, min(args.cpu_sample_grid_rows, g))
    es = np.dtype(dt).itemsize
    flops = float(n) * g * g  # sum over rows of b^2 / 2 multiply-add pairs, x 2
    band_bytes = float(es) * n * (g + 1)
    _lib.stage_timing(True)
    for order in args.orders.split(","):
        cold = None
        if order == "nd":
            # cold: a fresh handle (uploaded first, outside the clock), so the
            # host analysis (graph, bisection, symbolic) and the plan upload
            # are in the timed call; the warm calls below reuse the handle's plan
            A_cold = Csr.from_csr_arrays((n, n), rp, ci, v)
            A_cold._device()
            t0 = time.perf_counter()
            solve(A_cold, B, order=order)
            cold = {"wall_ms": round(1e3 * (time.perf_counter() - t0), 2),
                    "stages_ms": {k: round(t, 3) for k, t in _lib.stage_times().items()}}
            del A_cold
        solve(A, B, order=order)  # warm-up (first call uploads A; nd: builds the plan)
        walls, stages = [], []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            x = solve(A, B, order=order).get_col(0)
            walls.append(time.perf_counter() - t0)
            stages.append(_lib.stage_times())
        st = {k: round(float(np.mean([s[k] for s in stages])), 3) for k in stages[-1]}
        if order == "nd":  # the nested-dissection stages under the common names (the band flop model does not apply)
            st = {{"nd_factor": "cholesky", "nd_forward": "forward", "nd_backward": "backward"}.get(k, k): t
                  for k, t in st.items()}
        rel = float(np.linalg.norm(x.astype(np.float64) - x_true) / np.linalg.norm(x_true))
        line = {
            "metric": "C5 solve: device ms per stage, flop/byte roofline per kernel",
            "config": {"workload": f"c5: 2D 5-point Poisson {g}x{g} (N={n:,}, band {g}), natural ordering, "
                                   f"b = A x_true (seed 1002), 1 RHS", "dtype": args.dtype, "order": order},
            "wall_ms": round(1e3 * float(np.median(walls)), 2),
            "stages_ms": st,
            "device_ms_total": round(sum(st.values()), 2),
            "factor": {"kernel": {"reference": f"{band_kernel()} (reference order)", "blocked": "blk_chol (blocked)",
                                  "nd": "nd_factor (multifrontal, nested dissection; band flop count for scale only)"}[order],
                       "flops": flops, "ms": st.get("cholesky"),
                       "achieved_TFs": round(flops / (st["cholesky"] * 1e-3) / 1e12, 3) if st.get("cholesky") else None,
                       "peak_TFs": F64_PEAK_TFS,
                       "frac": round(flops / (st["cholesky"] * 1e-3) / 1e12 / F64_PEAK_TFS, 5)
                       if st.get("cholesky") else None},
            "forward": {"bytes": band_bytes, "ms": st.get("forward"),
                        "achieved_GBs": round(band_bytes / (st["forward"] * 1e-3) / 1e9, 1) if st.get("forward") else None,
                        "peak_GBs": HBM_PEAK_GBS,
                        "frac": round(band_bytes / (st["forward"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
                        if st.get("forward") else None},
            "backward": {"bytes": band_bytes, "ms": st.get("backward"),
                         "achieved_GBs": round(band_bytes / (st["backward"] * 1e-3) / 1e9, 1) if st.get("backward") else None,
                         "peak_GBs": HBM_PEAK_GBS,
                         "frac": round(band_bytes / (st["backward"] * 1e-3) / 1e9 / HBM_PEAK_GBS, 5)
                         if st.get("backward") else None},
            "cold": cold,
            "rel_err_vs_x_true": rel,
            "cpu_baseline": cpu,
            "vs_cpu": round(cpu["value_s"] / (float(np.median(walls))), 1) if cpu else None,
        }
        if fixture is not None:
            h = hashlib.sha256(np.ascontiguousarray(x, dtype=np.float64).view(np.uint64).tobytes()).hexdigest()
            line["x_bits_equal_oracle_fixture"] = h == fixture["sha256_x_f64_bits"]
            ex = np.array([int(t, 16) for t in fixture["x_sample_bits"]], dtype=np.uint64).view(np.float64)
            xs = x[::fixture["x_stride"]][:ex.size].astype(np.float64)
            line["max_rel_dev_vs_oracle_x_sample"] = float(np.max(np.abs(xs - ex) / np.abs(ex)))
            line["oracle_fixture_cpu_s"] = fixture.get("cpu_seconds")
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
