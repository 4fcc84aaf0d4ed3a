"""Helpers to read tests/golden/*.json (data transcribed from the reference's
#[test] functions). f32 literals are parsed with correct decimal -> f32
rounding, as rustc does for an f32 literal; [num, den] pairs are f32
divisions, as rustc constant-folds `(7.0/5.0)` in an f32 context."""

from __future__ import annotations

import json
import os
from fractions import Fraction

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))


def load(name: str = "reference_unit_tests.json") -> dict:
    with open(os.path.join(HERE, name)) as f:
        return json.load(f)


def _bits(x: np.float32) -> int:
    return int(np.asarray(x, dtype=np.float32).view(np.uint32))


def f32(s) -> np.float32:
    if isinstance(s, list):
        return np.float32(f32(s[0]) / f32(s[1]))
    x = Fraction(str(s))
    f = np.float32(float(x))
    cands = [np.nextafter(f, np.float32(-np.inf)), f, np.nextafter(f, np.float32(np.inf))]
    return min(cands, key=lambda c: (abs(Fraction(float(c)) - x), _bits(c) & 1))


def scalars(vals, dtype):
    dt = np.dtype(dtype)
    if dt == np.float32:
        return [f32(v) for v in vals]
    if dt.kind == "f":
        return [float(v) for v in vals]
    return [int(v) for v in vals]


def matrix(rows, dtype):
    """List-of-lists with every literal parsed for `dtype`."""
    return [scalars(r, dtype) for r in rows]
