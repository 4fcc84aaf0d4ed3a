"""Dense<T> (reference src/dense.rs:4-62): column-major, one array per column.

``Dense.new_default_with_dims(col_count, row_count)`` takes COLUMNS FIRST
(dense.rs:13) and ``Dense.from_data`` takes a list of COLUMNS (dense.rs:21-29)
-- the opposite of ``Csr.from_data``'s rows.
"""

from __future__ import annotations

import numpy as np

from .util import GetDims, MatDim


def _infer_dtype(values, dtype):
    if dtype is not None:
        return np.dtype(dtype)
    a = np.asarray(values)
    if a.dtype.kind == "f":
        return np.dtype(np.float64)  # Rust float literal default
    if a.dtype.kind in "iub":
        return np.dtype(np.int32)  # Rust integer literal default
    return a.dtype


class Dense(GetDims):
    __slots__ = ("col_count", "row_count", "data")

    def __init__(self, col_count: int, row_count: int, data):
        self.col_count = int(col_count)
        self.row_count = int(row_count)
        self.data = data  # list of 1-D numpy arrays, one per column

    @property
    def dtype(self):
        return self.data[0].dtype if self.data else np.dtype(np.float64)

    @classmethod
    def new_default_with_dims(cls, col_count: int, row_count: int, dtype=np.float64) -> "Dense":
        """dense.rs:13-15 (T::default() everywhere)."""
        return cls.new_with_dims(np.dtype(dtype).type(0), col_count, row_count, dtype=dtype)

    @classmethod
    def new_with_dims(cls, val, col_count: int, row_count: int, dtype=None) -> "Dense":
        """dense.rs:17-19."""
        dt = _infer_dtype([val], dtype)
        return cls(col_count, row_count, [np.full(row_count, val, dtype=dt) for _ in range(col_count)])

    @classmethod
    def from_data(cls, data, dtype=None) -> "Dense":
        """dense.rs:21-29: ``data`` is a list of COLUMNS; row_count = len(data[0])."""
        dt = _infer_dtype([x for col in data for x in col] or [0.0], dtype)
        cols = [np.array(col, dtype=dt) for col in data]
        return cls(len(data), len(data[0]), cols)

    @classmethod
    def from_columns(cls, columns, dtype=None) -> "Dense":
        """Bulk constructor (this build's addition): adopt numpy columns."""
        dt = np.dtype(dtype) if dtype is not None else np.asarray(columns[0]).dtype
        cols = [np.ascontiguousarray(c, dtype=dt) for c in columns]
        return cls(len(cols), len(cols[0]) if cols else 0, cols)

    def get_col(self, col_index: int) -> np.ndarray:
        """dense.rs:31-33 (read-only view)."""
        v = self.data[col_index].view()
        v.flags.writeable = False
        return v

    def get_col_mut(self, col_index: int) -> np.ndarray:
        """dense.rs:35-37 (writable)."""
        return self.data[col_index]

    def get_dims(self) -> MatDim:
        """dense.rs:40-47."""
        return MatDim(rows=self.row_count, cols=self.col_count)

    def __eq__(self, other) -> bool:  # derived PartialEq (dense.rs:4)
        if not isinstance(other, Dense):
            return NotImplemented
        if (self.col_count, self.row_count, len(self.data)) != (other.col_count, other.row_count, len(other.data)):
            return False
        return all(a.shape == b.shape and bool(np.all(a == b)) for a, b in zip(self.data, other.data))

    def __repr__(self) -> str:
        return f"Dense {{ col_count: {self.col_count}, row_count: {self.row_count}, data: {[list(c) for c in self.data]} }}"

    def __str__(self) -> str:  # dense.rs:49-62
        out = []
        for r in range(self.row_count):
            out.append("|" + "".join(f"{self.data[c][r]!s:>5}" for c in range(self.col_count)) + "|")
        return "\n".join(out) + ("\n" if out else "")
