#!/usr/bin/env python3
"""Generate tests/golden/c5_poisson_1000.json: the band oracle's exact C5
result (2D Poisson, 1000 x 1000 grid, N = 1M, bandwidth 1000, f64), so the
GPU's exact solve can be pinned bit for bit at full size.

BUILD CONTAINER ONLY (≈30-40 min of one CPU core, ≈35 GB of RAM). The chain
is the oracle's restatement of solve (src/lib.rs:11-24):
  L  = cholesky_decomp(A)   band restatement of sparse.rs:682-714
  L* = transpose(L)         sparse.rs:296-318
  y  = forward_substitution(L, b)    lib.rs:28-46
  x  = backward_substitution(L*, y)  lib.rs:49-65
with b = A x_true (x_true from seed 1002, b summed per row in entry order
from 0.0 exactly as tests/test_gpu_solver.py forms it).

The fixture holds hashes and strided samples only (a few hundred KB):
SHA-256 of x's f64 bits, of L's value bits / column indices / row_ptr, a
strided sample of x, a handful of full L rows, and nnz(L).
"""

from __future__ import annotations

import hashlib
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from oracle import pyoracle as orc  # noqa: E402

OUT = os.path.join(ROOT, "tests", "golden", "c5_poisson_1000.json")
G = 1000
SAMPLE_ROWS = [0, 1, 999, 1000, 1001, 123_456, 500_000, 999_000, 999_999]
X_STRIDE = 997


def sha(a) -> str:
    return hashlib.sha256(np.ascontiguousarray(a).tobytes()).hexdigest()


def log(msg):
    print(f"[c5-fixture {time.strftime('%H:%M:%S')}] {msg}", flush=True)


def rhs(rp, ci, v, n):
    """b = A x_true, per row in entry order starting from 0.0 (np.add.at is
    an unbuffered in-order accumulation)."""
    x_true = orc.gen_x_cols(1002, n, 1)[0]
    rows = np.repeat(np.arange(n), np.diff(rp.astype(np.int64)))
    b = np.zeros(n)
    np.add.at(b, rows, v * x_true[ci.astype(np.int64)])
    return x_true, b


def main():
    n = G * G
    rp, ci, v = orc.poisson2d(G)
    x_true, b = rhs(rp, ci, v, n)
    log(f"A: n={n} nnz={len(v)}; b sha {sha(b)[:16]}")
    t0 = time.time()
    lrp, lci, lv = orc.cholesky(n, n, rp, ci, v, band=True)
    t_chol = time.time() - t0
    log(f"L: nnz={len(lv)} in {t_chol:.0f} s")
    lrp64 = lrp.astype(np.int64)
    rows = {}
    for r in SAMPLE_ROWS:
        s, e = int(lrp64[r]), int(lrp64[r + 1])
        rows[str(r)] = {"cols": lci[s:e].astype(np.int64).tolist(),
                        "bits": [f"{u:016x}" for u in lv[s:e].view(np.uint64).tolist()]}
    l_fix = {"nnz": int(len(lv)), "sha256_row_ptr_i64": sha(lrp64), "sha256_col_i64": sha(lci.astype(np.int64)),
             "sha256_val_f64_bits": sha(lv), "rows": rows}
    t0 = time.time()
    urp, uci, uv = orc.transpose(n, n, lrp, lci, lv)
    t_tr = time.time() - t0
    log(f"L*: {t_tr:.0f} s")
    t0 = time.time()
    y = orc.forward_substitution(n, lrp, lci, lv, [b])
    t_fw = time.time() - t0
    del lrp, lci, lv
    t0 = time.time()
    x = orc.backward_substitution(n, urp, uci, uv, y)[0]
    t_bw = time.time() - t0
    log(f"forward {t_fw:.0f} s, backward {t_bw:.0f} s")
    rel = float(np.linalg.norm(x - x_true) / np.linalg.norm(x_true))
    fix = {
        "what": "band-oracle solve of C5 (2D Poisson 1000x1000, natural order, f64), b = A x_true(seed 1002)",
        "generator": "scripts/make_c5_fixture.py (oracle/bsm_oracle_tpl.inc: orc_cholesky_band_f64, "
                     "orc_transpose_f64, orc_forward_substitution_f64, orc_backward_substitution_f64)",
        "reference": "src/lib.rs:11-65, src/sparse.rs:296-318, 682-714",
        "g": G, "n": n,
        "sha256_b_f64_bits": sha(b),
        "sha256_y_f64_bits": sha(y[0]),
        "sha256_x_f64_bits": sha(x),
        "x_stride": X_STRIDE,
        "x_sample_bits": [f"{u:016x}" for u in x[::X_STRIDE].view(np.uint64).tolist()],
        "rel_err_vs_x_true": rel,
        "L": l_fix,
        "cpu_seconds": {"cholesky_band_two_passes": round(t_chol, 1), "transpose": round(t_tr, 1),
                        "forward": round(t_fw, 1), "backward": round(t_bw, 1)},
    }
    with open(OUT, "w") as f:
        json.dump(fix, f, indent=1)
    log(f"wrote {OUT} (rel err vs x_true {rel:.3e})")


if __name__ == "__main__":
    main()
