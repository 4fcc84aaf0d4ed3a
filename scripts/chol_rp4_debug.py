#!/usr/bin/env python3
"""Locate the first wrong entry of an A/B band_chol5 build's factor against
the band oracle's (plain C, test infrastructure), in dependency order
(row-block, then column),
and print the pattern of wrong entries in that row-block: which of its 16 rows
(and so which wave: rows RP*w .. RP*w + RP - 1), which columns (tile K =
col // 16, slot m = (col - jb) // 64, lane = (col - jb) % 64), and the values.

  BSM_LIB_PATH=basic_sparse_matrix_amd/lib/libbsm_hip_rp4.so \
      python scripts/chol_rp4_debug.py --g 500 --rpw 4

Diagnostic only (the band_chol5 RP = 4 wrong-bits investigation, round 5;
the A/B build: scripts/perf/build_rp4.sh).
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
import numpy as np  # noqa: E402

from basic_sparse_matrix_amd import Csr  # noqa: E402
from oracle import pyoracle as orc  # noqa: E402  (the input matrix only)


def factor(A, rpw=None):
    if rpw:
        os.environ["BSM_CHOL_RPW"] = str(rpw)
    else:
        os.environ.pop("BSM_CHOL_RPW", None)
    L = A.cholesky_decomp()
    out = (np.asarray(L.row_index).astype(np.int64).copy(), np.asarray(L.col_index).astype(np.int64).copy(),
           np.asarray(L.v).copy())
    del L
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--g", type=int, default=500)
    ap.add_argument("--rpw", type=int, default=4)
    ap.add_argument("--reps", type=int, default=2)
    ap.add_argument("--show", type=int, default=40)
    a = ap.parse_args()
    n = a.g * a.g
    rp, ci, v = orc.poisson2d(a.g)
    A = Csr.from_csr_arrays((n, n), rp, ci, v)
    erp, eci, ev = orc.cholesky(n, n, rp, ci, v, band=True)
    ref = (np.asarray(erp).astype(np.int64), np.asarray(eci).astype(np.int64), np.asarray(ev))
    b = a.g  # Poisson 2D bandwidth
    for rep in range(a.reps):
        got = factor(A, a.rpw)
        res = {"g": a.g, "rpw": a.rpw, "rep": rep, "lib": os.environ.get("BSM_LIB_PATH", "default")}
        if not (np.array_equal(ref[0], got[0]) and np.array_equal(ref[1], got[1])):
            res["structure_differs"] = True
            print(json.dumps(res), flush=True)
            continue
        rv, gv = ref[2], got[2]
        bad = np.nonzero(rv.view(np.uint64) != gv.view(np.uint64))[0]
        res["values_differing"] = int(bad.size)
        if bad.size == 0:
            print(json.dumps(res), flush=True)
            continue
        rows = np.searchsorted(ref[0], bad, side="right") - 1
        cols = ref[1][bad]
        order = np.lexsort((cols, rows // 16))
        I = int(rows[order[0]] // 16)
        i0 = 16 * I
        K0 = max(i0 - b, 0) // 16
        jb = 16 * K0
        sel = order[rows[order] // 16 == I]
        res.update({"first_row_block": I, "K0": K0, "jb": jb, "wrong_in_block": int(sel.size)})
        first = []
        for p in sel[: a.show]:
            r, c = int(rows[p]), int(cols[p])
            first.append({"row": r, "r_in_block": r - i0, "wave": (r - i0) // a.rpw, "col": c, "tile": c // 16,
                          "slot": (c - jb) // 64, "lane": (c - jb) % 64, "ref": float(rv[bad[p]]),
                          "got": float(gv[bad[p]])})
        res["first"] = first
        # wrong (row-in-block, tile) pairs in the first bad row-block
        pairs = sorted({(int(rows[p]) - i0, int(cols[p]) // 16) for p in sel})
        res["rows_wrong"] = sorted({p[0] for p in pairs})
        res["tiles_wrong_first_row"] = sorted({p[1] for p in pairs if p[0] == res["rows_wrong"][0]})[:20]
        # row-blocks with any wrong value (first 40)
        res["row_blocks_wrong"] = sorted(set((rows // 16).tolist()))[:40]
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
