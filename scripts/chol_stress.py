#!/usr/bin/env python3
"""Repeat the band Cholesky of the g x g Poisson matrix with several kernel
variants and compare every factor bit for bit with the first band_chol4 one
(BSM_CHOL_VARIANT=4), to catch ordering races that a single run can miss.

  python scripts/chol_stress.py --g 500 --reps 4 --variants 4 5:4 5:2

A variant is BSM_CHOL_VARIANT[:BSM_CHOL_RPW]. Prints one JSON line per
variant: runs, mismatching runs, and for the first mismatch the number of
differing values and the first differing row.
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


def factor(A, variant):
    v, _, rpw = variant.partition(":")
    os.environ["BSM_CHOL_VARIANT"] = v
    if rpw:
        os.environ["BSM_CHOL_RPW"] = rpw
    else:
        os.environ.pop("BSM_CHOL_RPW", None)
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
    ap.add_argument("--variants", nargs="+", default=["4", "5:4", "5:2"])
    a = ap.parse_args()
    n = a.g * a.g
    rp, ci, v = orc.poisson2d(a.g)
    A = Csr.from_csr_arrays((n, n), rp, ci, v)
    ref, _ = factor(A, "4")
    for var in a.variants:
        bad, first, times = 0, None, []
        for _ in range(a.reps):
            got, dt = factor(A, var)
            times.append(round(dt * 1e3, 1))
            same = all(np.array_equal(x, y) for x, y in zip(ref, got))
            if not same:
                bad += 1
                if first is None and np.array_equal(ref[0], got[0]):
                    diff = np.nonzero(ref[2] != got[2])[0]
                    row = int(np.searchsorted(ref[0].astype(np.int64), diff[0], side="right") - 1)
                    first = {"values_differing": int(diff.size), "first_row": row, "first_row_block": row // 16}
        print(json.dumps({"g": a.g, "variant": var, "lib": os.environ.get("BSM_LIB_PATH", "default"), "runs": a.reps,
                          "mismatching_runs": bad, "first_mismatch": first, "ms": times}), flush=True)


if __name__ == "__main__":
    main()
