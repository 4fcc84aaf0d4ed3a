"""Linear solver of the reference crate (src/lib.rs:11-65), on the GPU.

``solve(a, b)`` = cholesky_decomp -> transpose -> forward_substitution ->
backward_substitution, with the reference's exact operation order
(DESIGN.md "Solver"). The reference is ``f32``-only; ``f64`` is accepted as
this build's addition.
"""

from __future__ import annotations

import numpy as np

from . import _lib
from .dense import Dense
from .sparse import Csr, _raise_for
from .util import Panic

_FLOATS = (np.dtype(np.float32), np.dtype(np.float64))


def _check_types(m: Csr, d: Dense, what: str):
    if m.dtype not in _FLOATS or d.dtype != m.dtype:
        raise TypeError(f"{what}: needs Csr<f32>/Dense<f32> (or f64), got {m.dtype}/{d.dtype}")


def _run(fn_name: str, m: Csr, rhs: Dense) -> Dense:
    dims = rhs.get_dims()
    n, k = dims.rows, dims.cols
    if m.dims.rows < n:
        raise Panic("index out of bounds: matrix has fewer rows than the right-hand side")
    b_cols = []
    for j in range(k):
        c = np.ascontiguousarray(rhs.get_col(j))
        if c.shape[0] < n:  # b.get_col(c)[row] / y.get_col(c)[row] for every row < n (lib.rs:33, :54)
            raise Panic(f"index out of bounds: the len is {c.shape[0]} but the index is {c.shape[0]}")
        b_cols.append(np.ascontiguousarray(c[:n]))
    dev = m._device()
    lib = _lib.require_device()
    out = Dense.new_default_with_dims(k, n, dtype=m.dtype)
    _raise_for(getattr(lib, fn_name)(dev.handle, k, n, _lib.ptr_array(b_cols), _lib.ptr_array(out.data)))
    return out


def forward_substitution(l: Csr, b: Dense) -> Dense:
    """lib.rs:28-46: solve L y = b (diagonal = LAST stored entry of each row)."""
    _check_types(l, b, "forward_substitution")
    return _run("bsm_forward_substitution", l, b)


def backward_substitution(l_star: Csr, y: Dense) -> Dense:
    """lib.rs:49-65: solve L* x = y (diagonal = FIRST stored entry of each row)."""
    _check_types(l_star, y, "backward_substitution")
    return _run("bsm_backward_substitution", l_star, y)


def solve(a: Csr, b: Dense, *, order: str = "reference") -> Dense:
    """lib.rs:11-24. Non-square ``a`` panics (``cholesky_decomp().unwrap()``).

    ``order="reference"`` (default) keeps the reference's operation order:
    bit-exact. ``order="blocked"`` reassociates the two triangular solves
    (64-row blocks, precomputed inverse diagonal blocks; ``bsm_solve_blocked``):
    not bit-exact, within the north star's 1e-6 relative f64 tolerance, and
    ~100x faster on C5's triangular solves. This keyword is this build's
    addition; the reference has one order."""
    _check_types(a, b, "solve")
    if a.dims.rows != a.dims.cols:
        raise Panic("called `Result::unwrap()` on an `Err` value: NonSquareMatrix")
    if order not in ("reference", "blocked"):
        raise ValueError(f"solve: order must be 'reference' or 'blocked', got {order!r}")
    return _run("bsm_solve" if order == "reference" else "bsm_solve_blocked", a, b)
