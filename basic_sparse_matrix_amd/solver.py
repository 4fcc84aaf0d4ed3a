"""Linear solver of the reference crate (src/lib.rs:11-65), on the GPU.

``solve(a, b)`` = cholesky_decomp -> transpose -> forward_substitution ->
backward_substitution, with the reference's exact operation order
(DESIGN.md "Solver"). The reference is ``f32``-only; ``f64`` is accepted as
this build's addition.
"""

from __future__ import annotations

import ctypes

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
    addition; the reference has one order.

    ``order="nd"`` factors P A P^T instead, P a nested-dissection order of
    A's graph (``bsm_solve_nd``: the host bisects the graph, the device
    factors the separator tree's dense fronts level by level): a wide
    elimination tree with far fewer flops than the band on 2-D meshes; also
    within the 1e-6 relative f64 tolerance, not bit-exact."""
    _check_types(a, b, "solve")
    if a.dims.rows != a.dims.cols:
        raise Panic("called `Result::unwrap()` on an `Err` value: NonSquareMatrix")
    fns = {"reference": "bsm_solve", "blocked": "bsm_solve_blocked", "nd": "bsm_solve_nd"}
    if order not in fns:
        raise ValueError(f"solve: order must be 'reference', 'blocked' or 'nd', got {order!r}")
    return _run(fns[order], a, b)


def nd_analyse(n: int, row_ptr, col_idx, leaf: int = 256) -> dict:
    """The host analysis of ``solve(order="nd")`` on a CSR pattern
    (``bsm_nd_analyse``; no device): ``perm`` (perm[new] = old) and the
    separator tree in post-order (``start``, ``end``, ``parent``, ``level``,
    ``slot``, front rows ``st``)."""
    lib = _lib.load()
    rp = np.ascontiguousarray(row_ptr, dtype=np.uint64)
    ci = np.ascontiguousarray(col_idx, dtype=np.uint64)
    perm = np.zeros(n, dtype=np.int64)
    nn = ctypes.c_uint64(0)
    sl = ctypes.c_uint64(0)
    _lib.check(lib.bsm_nd_analyse(n, _lib.ptr(rp), _lib.ptr(ci), leaf, _lib.ptr(perm), None, 0, ctypes.byref(nn),
                                  None, 0, ctypes.byref(sl)))
    nodes = np.zeros((max(nn.value, 1), 8), dtype=np.int64)
    st = np.zeros(max(sl.value, 1), dtype=np.int64)
    _lib.check(lib.bsm_nd_analyse(n, _lib.ptr(rp), _lib.ptr(ci), leaf, _lib.ptr(perm), _lib.ptr(nodes), nn.value,
                                  ctypes.byref(nn), _lib.ptr(st), sl.value, ctypes.byref(sl)))
    nodes = nodes[: nn.value]
    return {"perm": perm, "start": nodes[:, 0], "end": nodes[:, 1], "parent": nodes[:, 2], "level": nodes[:, 3],
            "slot": nodes[:, 4],
            "st": [st[o: o + m] for m, o in zip(nodes[:, 5], nodes[:, 6])]}
