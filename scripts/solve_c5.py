#!/usr/bin/env python3
"""C5 (north_star config 5): 2D 5-point Poisson on a g x g grid (natural
ordering, N = g^2, band b = g), b = A x_true, solve(A, b) on the GPU through
the reference API (lib.rs:11-24): cholesky_decomp -> transpose -> forward ->
backward substitution. Prints ONE JSON line per order (reference = bit-exact
operation order; blocked = reassociated, within 1e-6 on f64) with

* wall time through the public API (host b in, host x out) and the device
  time of every stage (HIP events on the library's stream, bsm_stage_times);
* the band orders: the factor's flop roofline (N b^2 flops, the band
  Cholesky's multiply-add pairs x 2, against the 78.6 TF/s f64 peak of
  MI355X_MICROARCH.md) and each triangular solve's byte roofline (the band
  of L, 8 N (b+1) bytes, read once, against 8 TB/s);
* the nd order: its own model from its plan (nd_model: the fronts' true and
  64-padded flops, the bytes of its L), never the band's; the cold figure
  (first solve of the pattern, new handle, analysis included) first, since
  solve(a, b) takes `a` by value (lib.rs:11), then new handles of a pattern
  seen before (the plan from the library's cache), then the same handle;
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

from basic_sparse_matrix_amd import Csr, Dense, _lib, solve, solver  # noqa: E402
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


def nd_model(n, rp, ci, leaf, es):
    """The nested-dissection solve's own work model, from its plan (the host
    analysis alone, solver.nd_analyse, the same call the library makes):
    per front np pivots and m front rows.
    * true flops: sum of np^3/3 + np^2 m + np m^2 (the partial Cholesky of
      the front: its pivot block, the panel below it, the update block);
    * padded flops: what nd_factor executes on 64 x 64 tiles (np padded to
      np_pad = 64 npt, nt = ceil((np_pad + m) / 64) tile rows): per lower
      tile (I, K) min(K, npt) tile products of 2 * 64^3, plus for a pivot
      column the diagonal tile's factor and inverse (2 * 64^3 / 3) or the
      sub-diagonal tile's product with the inverse (2 * 64^3);
    * L bytes: es * (np (np + 1) / 2 + np m) over the fronts, the entries of
      L each triangular solve must read once (the algorithmic bytes), and the
      padded bytes the solve kernels read (the pivot columns' lower tiles and
      the inverse diagonal tiles)."""
    plan = solver.nd_analyse(n, rp, ci, leaf=leaf)
    npv = (plan["end"] - plan["start"]).astype(np.float64)
    m = np.array([len(x) for x in plan["st"]], dtype=np.float64)
    true_flops = float(np.sum(npv ** 3 / 3 + npv ** 2 * m + npv * m ** 2))
    npt = np.ceil(npv / 64)
    nt = np.ceil((64 * npt + m) / 64)
    t3 = 64.0 ** 3
    padded = 0.0
    solve_bytes = 0.0
    for p_, q_ in zip(npt.astype(np.int64), nt.astype(np.int64)):
        # products: tiles (I, K), K < nt, I >= K, each min(K, npt) products
        ks = np.arange(q_)
        padded += 2 * t3 * float(np.sum((q_ - ks) * np.minimum(ks, p_)))
        padded += p_ * 2 * t3 / 3 + 2 * t3 * float(np.sum(q_ - 1 - np.arange(p_)))
        solve_bytes += es * 4096.0 * (float(np.sum(q_ - 1 - np.arange(p_))) + p_)
    l_bytes = float(es * np.sum(npv * (npv + 1) / 2 + npv * m))
    return {"leaf": leaf, "fronts": int(npv.size), "true_flops": true_flops, "padded_flops": padded,
            "l_bytes": l_bytes, "padded_solve_bytes": solve_bytes,
            "l_nnz": int(np.sum(npv * (npv + 1) / 2 + npv * m))}


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


def roof(work, ms, peak, scale):
    """achieved (work / time, in the unit of `peak`) and its fraction of peak"""
    if not ms:
        return None, None
    a = work / (ms * 1e-3) / scale
    return round(a, 3), round(a / peak, 5)


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
        cold = by_value = model = nd_solves = None
        if order == "nd":
            leaf = int(os.environ.get("BSM_ND_LEAF", "192"))
            model = nd_model(n, rp, ci, leaf, es)
            # the process's first GPU work (runtime and device set-up, code
            # objects) on a small system of another pattern, outside the clock:
            # "cold" is the first solve of THIS pattern, not the process's first
            wrp, wci, wv = orc.poisson2d(16)
            solve(Csr.from_csr_arrays((256, 256), wrp, wci, wv.astype(dt)),
                  Dense.from_columns([np.ones(256, dtype=dt)]), order="nd")
            nd_solves = {"small_warmup_16x16": 1, "full": 1 + max(args.reps, 1) + 1 + args.reps}
            # cold: the first solve of this pattern in the process, as the
            # reference's solve(a, b) is called (lib.rs:11, `a` by value): a new
            # handle (uploaded inside the clock), the host analysis, the plan
            # upload, the first allocation of the fronts, the solve
            _lib.nd_cache_clear()
            t0 = time.perf_counter()
            A_cold = Csr.from_csr_arrays((n, n), rp, ci, v)
            A_cold._device()
            t_up = time.perf_counter()
            solve(A_cold, B, order=order)
            t1 = time.perf_counter()
            cold = {"wall_ms": round(1e3 * (t1 - t0), 2), "upload_ms": round(1e3 * (t_up - t0), 2),
                    "solve_call_ms": round(1e3 * (t1 - t_up), 2),
                    "stages_ms": {k: round(t, 3) for k, t in _lib.stage_times().items()}}
            del A_cold
            # by value, pattern seen before: a new handle per call again, the
            # plan found in the library's cache by the pattern
            walls, calls, st_bv = [], [], []
            for _ in range(max(args.reps, 1)):
                t0 = time.perf_counter()
                A_bv = Csr.from_csr_arrays((n, n), rp, ci, v)
                A_bv._device()
                t_up = time.perf_counter()
                solve(A_bv, B, order=order)
                t1 = time.perf_counter()
                walls.append(t1 - t0)
                calls.append(t1 - t_up)
                st_bv.append(_lib.stage_times())
                del A_bv
            by_value = {"wall_ms": round(1e3 * float(np.median(walls)), 2),
                        "solve_call_ms": round(1e3 * float(np.median(calls)), 2),
                        "upload_ms": round(1e3 * float(np.median(walls) - np.median(calls)), 2),
                        "stages_ms": {k: round(float(np.mean([s_[k] for s_ in st_bv])), 3) for k in st_bv[-1]},
                        "cache": _lib.nd_cache_info()}
        solve(A, B, order=order)  # warm-up (first call uploads A; nd: attaches the plan to the handle)
        walls, stages = [], []
        for _ in range(args.reps):
            t0 = time.perf_counter()
            x = solve(A, B, order=order).get_col(0)
            walls.append(time.perf_counter() - t0)
            stages.append(_lib.stage_times())
        st = {k: round(float(np.mean([s[k] for s in stages])), 3) for k in stages[-1]}
        rel = float(np.linalg.norm(x.astype(np.float64) - x_true) / np.linalg.norm(x_true))
        line = {
            "metric": "C5 solve: device ms per stage, flop/byte roofline per kernel",
            "config": {"workload": f"c5: 2D 5-point Poisson {g}x{g} (N={n:,}, band {g}), natural ordering, "
                                   f"b = A x_true (seed 1002), 1 RHS", "dtype": args.dtype, "order": order},
            "wall_ms": round(1e3 * float(np.median(walls)), 2),
            "stages_ms": st,
            "device_ms_total": round(sum(st.values()), 2),
        }
        if order == "nd":
            # scored against the nd plan's own work (nd_model), never the band's
            fms, fw, bw = st.get("nd_factor"), st.get("nd_forward"), st.get("nd_backward")
            ta, tf = roof(model["true_flops"], fms, F64_PEAK_TFS, 1e12)
            pa, pf = roof(model["padded_flops"], fms, F64_PEAK_TFS, 1e12)
            # one right-hand side with the pull: the forward solve is folded into
            # the factor's diagonal tiles (BSM_ND_FOLD), its stage only marks time
            folded = os.environ.get("BSM_ND_FOLD", "1") != "0" and os.environ.get("BSM_ND_PULL", "1") != "0"
            fa, ff = (None, None) if folded else roof(model["l_bytes"], fw, HBM_PEAK_GBS, 1e9)
            ba, bf = roof(model["l_bytes"], bw, HBM_PEAK_GBS, 1e9)
            line.update({
                "primary": "cold: solve(a, b) takes a by value (lib.rs:11), so a drop-in caller's first solve of "
                           "a pattern pays the analysis; by_value: later calls with new handles of that pattern; "
                           "wall_ms: the same handle again",
                "cold": cold, "by_value": by_value, "model": model, "nd_solves_in_process": nd_solves,
                "factor": {"stage": "nd_factor (zero tiles + assemble are nd_assemble; the extend-adds run inside "
                                    "this stage, so its time bounds the factor kernels' from above"
                                    + ("; the forward solve is folded into it" if folded else "") + ")",
                           "ms": fms, "true_flops": model["true_flops"], "padded_flops": model["padded_flops"],
                           "achieved_TFs_true": ta, "frac_true": tf, "achieved_TFs_padded": pa, "frac_padded": pf,
                           "peak_TFs": F64_PEAK_TFS},
                "forward": ({"ms": fw, "folded": "into nd_factor's diagonal tiles (BSM_ND_FOLD): y and the update "
                                                "vectors formed from the L tiles the factor holds; no pass over L"}
                            if folded else
                            {"ms": fw, "alg_bytes": model["l_bytes"], "padded_bytes_read": model["padded_solve_bytes"],
                             "achieved_GBs": fa, "frac": ff, "peak_GBs": HBM_PEAK_GBS}),
                "backward": {"ms": bw, "alg_bytes": model["l_bytes"], "padded_bytes_read": model["padded_solve_bytes"],
                             "achieved_GBs": ba, "frac": bf, "peak_GBs": HBM_PEAK_GBS},
            })
        else:
            fa, ff = roof(flops, st.get("cholesky"), F64_PEAK_TFS, 1e12)
            wa, wf = roof(band_bytes, st.get("forward"), HBM_PEAK_GBS, 1e9)
            ba, bf = roof(band_bytes, st.get("backward"), HBM_PEAK_GBS, 1e9)
            line.update({
                "factor": {"kernel": {"reference": f"{band_kernel()} (reference order)",
                                      "blocked": "blk_chol (blocked)"}[order],
                           "flops": flops, "ms": st.get("cholesky"), "achieved_TFs": fa, "peak_TFs": F64_PEAK_TFS,
                           "frac": ff},
                "forward": {"bytes": band_bytes, "ms": st.get("forward"), "achieved_GBs": wa,
                            "peak_GBs": HBM_PEAK_GBS, "frac": wf},
                "backward": {"bytes": band_bytes, "ms": st.get("backward"), "achieved_GBs": ba,
                             "peak_GBs": HBM_PEAK_GBS, "frac": bf},
            })
        line.update({
            "rel_err_vs_x_true": rel,
            "cpu_baseline": cpu,
            "vs_cpu": round(cpu["value_s"] / (float(np.median(walls))), 1) if cpu else None,
            "vs_cpu_cold": round(cpu["value_s"] / (cold["wall_ms"] * 1e-3), 1) if cpu and cold else None,
        })
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
