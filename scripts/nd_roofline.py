#!/usr/bin/env python3
"""The nd solve's kernels against their own rooflines, from a rocprofv3
kernel-stats CSV (--kernel-trace --stats of scripts/solve_c5.py --orders nd)
and the plan's work model in that run's JSON line (scripts/solve_c5.py's
"model": true / padded flops of the fronts, bytes of L).

Per solve (solves: the line's nd_solves_in_process["full"], else the calls
of nd_scatter, one per solve):
* factor: nd_factor's time; true flops and 64-padded flops against the
  78.6 TF/s FP64 MFMA peak (MI355X_MICROARCH.md);
* forward: nd_forward + nd_forward_tiles (none when the forward solve is
  folded into nd_factor, one right-hand side); backward: nd_backward +
  nd_backward_tiles; L's bytes (each entry read once) against 8 TB/s;
* the fixed costs beside them (zero tiles, assemble, extend-add).

usage: nd_roofline.py KERNEL_STATS.csv SOLVE_C5.jsonl [--dtype double] [--solves N]
"""
import argparse
import csv
import json

F64_PEAK_TFS = 78.6
HBM_PEAK_GBS = 8000.0


def kernel_ns(path, dtype):
    """{short kernel name: total ns} for the nd kernels of one dtype"""
    out = {}
    with open(path) as f:
        for row in csv.DictReader(f):
            name = row["Name"]
            for short in ("nd_factor", "nd_forward_tiles", "nd_forward", "nd_backward_tiles", "nd_backward",
                          "nd_zero_tiles", "nd_assemble", "nd_extend2", "nd_extend", "nd_pad_pivots", "nd_gather",
                          "nd_scatter", "nd_aent_vals", "nd_pattern_hash", "nd_pattern_diff"):
                # nd_factor<double, false>: the product instantiation (STAMPS off)
                if (f"{short}<{dtype}>" in name or f"{short}<{dtype}, false>" in name
                        or (short.startswith("nd_pattern") and f"{short}(" in name)):
                    out[short] = out.get(short, 0) + int(row["TotalDurationNs"])
                    out[short + ":calls"] = out.get(short + ":calls", 0) + int(row["Calls"])
                    break
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("csv")
    ap.add_argument("jsonl")
    ap.add_argument("--dtype", default="double")
    ap.add_argument("--solves", type=int, default=0,
                    help="full-size solves in the profiled run (a line without nd_solves_in_process)")
    args = ap.parse_args()
    model = nd_solves = None
    with open(args.jsonl) as f:
        for ln in f:
            ln = ln.strip()
            if ln.startswith("{"):
                d = json.loads(ln)
                if d.get("config", {}).get("order") == "nd":
                    model = d["model"]
                    nd_solves = d.get("nd_solves_in_process")
    assert model, "no nd line with a model in " + args.jsonl
    k = kernel_ns(args.csv, args.dtype)
    # the full-size solves of the run (solve_c5.py records them; its 16 x 16
    # warm-up solve's kernels stay in the totals: ~1 % of one C5 solve)
    solves = args.solves or (nd_solves or {}).get("full") or k.get("nd_scatter:calls", 0)
    assert solves > 0, "no nd_scatter calls in " + args.csv
    ms = lambda *names: sum(k.get(n, 0) for n in names) * 1e-6 / solves  # noqa: E731
    fac, fwd, bwd = ms("nd_factor"), ms("nd_forward", "nd_forward_tiles"), ms("nd_backward", "nd_backward_tiles")
    res = {
        "source": {"kernel_stats": args.csv, "model_from": args.jsonl, "solves": solves},
        "model": model,
        "factor": {"kernel": "nd_factor", "ms": round(fac, 4),
                   "achieved_TFs_true": round(model["true_flops"] / fac * 1e-9, 3),
                   "frac_true": round(model["true_flops"] / fac * 1e-9 / F64_PEAK_TFS, 4),
                   "achieved_TFs_padded": round(model["padded_flops"] / fac * 1e-9, 3),
                   "frac_padded": round(model["padded_flops"] / fac * 1e-9 / F64_PEAK_TFS, 4),
                   "peak_TFs": F64_PEAK_TFS},
        "forward": ({"kernels": "nd_forward + nd_forward_tiles", "ms": round(fwd, 4),
                     "achieved_GBs": round(model["l_bytes"] / fwd * 1e-6, 1),
                     "frac": round(model["l_bytes"] / fwd * 1e-6 / HBM_PEAK_GBS, 4), "peak_GBs": HBM_PEAK_GBS}
                    if fwd > 0 else
                    {"kernels": "none: folded into nd_factor's diagonal tiles (BSM_ND_FOLD)", "ms": 0.0}),
        "backward": {"kernels": "nd_backward + nd_backward_tiles", "ms": round(bwd, 4),
                     "achieved_GBs": round(model["l_bytes"] / bwd * 1e-6, 1),
                     "frac": round(model["l_bytes"] / bwd * 1e-6 / HBM_PEAK_GBS, 4), "peak_GBs": HBM_PEAK_GBS},
        "fixed_ms_per_solve": {n: round(ms(n), 4) for n in ("nd_zero_tiles", "nd_assemble", "nd_pad_pivots",
                                                            "nd_aent_vals", "nd_extend2", "nd_extend", "nd_gather",
                                                            "nd_scatter")
                               if k.get(n)},
    }
    for part in ("factor", "forward", "backward"):
        for key, val in res[part].items():
            if key.startswith("frac"):
                assert val <= 1.0, (part, key, val)
    print(json.dumps(res, indent=1))


if __name__ == "__main__":
    main()
