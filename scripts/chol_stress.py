#!/usr/bin/env python3
"""Repeat the band Cholesky (band_chol5) of the g x g Poisson matrix and
compare every factor bit for bit with the band oracle's (plain C, test
infrastructure: ~30 s at g = 500), to catch ordering races that a single run
can miss. A/B builds of the library go in by BSM_LIB_PATH (e.g. the RP = 4
build of scripts/perf/build_rp4.sh with --rpw 4).

  python scripts/chol_stress.py --g 500 --reps 4

Prints one JSON line: runs, mismatching runs, and for the first mismatch the
number of differing values and the first differing row.
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from basic_sparse_matrix_amd import Csr  # noqa: E402
from oracle import pyoracle as orc  # noqa: E402  (the input matrix only)


def factor(A, rpw):
    if rpw:
        os.environ["BSM_CHOL_RPW"] = str(rpw)
    t = time.perf_counter()
    L = A.cholesky_decomp()
    dt = time.perf_counter() - t
    out = (np.asarray(L.row_index).copy(), np.asarray(L.col_index).copy(), np.asarray(L.v).view(np.uint64).copy())
    del L
    return out, dt


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--g", type=int, default=500)
    ap.add_argument("--reps", type=int, default=4)
    ap.add_argument("--rpw", type=int, default=0, help="BSM_CHOL_RPW for an A/B build (0: leave unset)")
    a = ap.parse_args()
    n = a.g * a.g
    rp, ci, v = orc.poisson2d(a.g)
    A = Csr.from_csr_arrays((n, n), rp, ci, v)
    t = time.perf_counter()
    erp, eci, ev = orc.cholesky(n, n, rp, ci, v, band=True)
    oracle_s = time.perf_counter() - t
    ref = (np.asarray(erp, np.uint64), np.asarray(eci, np.uint64), np.asarray(ev).view(np.uint64))
    bad, first, times = 0, None, []
    for _ in range(a.reps):
        got, dt = factor(A, a.rpw)
        got = (got[0].astype(np.uint64), got[1].astype(np.uint64), got[2])
        times.append(round(dt * 1e3, 1))
        same = all(np.array_equal(x, y) for x, y in zip(ref, got))
        if not same:
            bad += 1
            if first is None and np.array_equal(ref[0], got[0]):
                diff = np.nonzero(ref[2] != got[2])[0]
                row = int(np.searchsorted(ref[0].astype(np.int64), diff[0], side="right") - 1)
                first = {"values_differing": int(diff.size), "first_row": row, "first_row_block": row // 16}
    print(json.dumps({"g": a.g, "rpw": a.rpw, "lib": os.environ.get("BSM_LIB_PATH", "default"), "runs": a.reps,
                      "mismatching_runs": bad, "first_mismatch": first, "ms": times,
                      "oracle_s": round(oracle_s, 1)}), flush=True)


if __name__ == "__main__":
    main()
