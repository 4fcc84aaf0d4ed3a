"""The C5 nd roofline record is reproducible from the committed files
(VERDICT r5 "next" item 1): scripts/nd_roofline.py recomputes the factor's and
the triangular solves' fractions from the rocprofv3 kernel-stats CSV and the
solve_c5.py line (the nd plan's own flop and byte model), every fraction is
at most 1, and the result equals the committed JSON. CPU only."""

import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PROF = os.path.join(ROOT, "profiles")


@pytest.mark.parametrize("tag", ["r06_c", "r06_o", "r06_w", "r06_x", "r06_z"])
def test_nd_roofline_reproducible(tag):
    csv_p = os.path.join(PROF, f"{tag}_c5_nd_kernel_stats.csv")
    jsonl_p = os.path.join(PROF, f"{tag}_solve_c5_nd_profiled.jsonl")
    committed = os.path.join(PROF, f"{tag}_nd_roofline.json")
    if not (os.path.exists(csv_p) and os.path.exists(jsonl_p) and os.path.exists(committed)):
        pytest.skip("profile files absent")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "scripts", "nd_roofline.py"),
                        os.path.relpath(csv_p, ROOT), os.path.relpath(jsonl_p, ROOT)],
                       capture_output=True, text=True, cwd=ROOT, timeout=60)
    assert r.returncode == 0, r.stderr
    got = json.loads(r.stdout)
    with open(committed) as f:
        want = json.load(f)
    for part in ("factor", "forward", "backward"):
        assert got[part] == want[part], part
        for k, v in got[part].items():
            if k.startswith("frac"):
                assert 0 < v <= 1, (part, k, v)
    # the band model is gone from the nd line: its own model, from its plan
    with open(jsonl_p) as f:
        line = [json.loads(x) for x in f if x.startswith("{")][-1]
    assert line["model"]["true_flops"] < 1e11 and line["factor"]["frac_true"] <= 1
    # the forward solve folded into the factor (one right-hand side) has no
    # pass, hence no fraction, of its own
    assert line["forward"].get("folded") or line["forward"]["frac"] <= 1
    assert line["backward"]["frac"] <= 1
