"""DenseS<T, ROWS, COLS> (reference src/dense_static.rs:4-68).

Rust's const generics become constructor arguments: ``DenseS.new_default(7, 5,
np.int32)`` is ``DenseS::<i32,7,5>::new_default()``. Storage is
``[[T; ROWS]; COLS]`` -> a (COLS, ROWS) array.
"""

from __future__ import annotations

import numpy as np

from .dense import _infer_dtype
from .util import GetDims, MatDim, Panic


class DenseS(GetDims):
    __slots__ = ("ROWS", "COLS", "col_count", "row_count", "data")

    def __init__(self, ROWS: int, COLS: int, col_count: int, row_count: int, data: np.ndarray):
        self.ROWS, self.COLS = int(ROWS), int(COLS)
        self.col_count, self.row_count = int(col_count), int(row_count)
        self.data = data

    @property
    def dtype(self):
        return self.data.dtype

    @classmethod
    def new_default(cls, ROWS: int, COLS: int, dtype=np.float64) -> "DenseS":
        """dense_static.rs:13-15."""
        return cls.new(np.dtype(dtype).type(0), ROWS, COLS, dtype)

    @classmethod
    def new(cls, val, ROWS: int, COLS: int, dtype=None) -> "DenseS":
        """dense_static.rs:17-19."""
        dt = _infer_dtype([val], dtype)
        return cls(ROWS, COLS, COLS, ROWS, np.full((COLS, ROWS), val, dtype=dt))

    @classmethod
    def from_data(cls, data, ROWS: int = None, COLS: int = None, dtype=None) -> "DenseS":
        """dense_static.rs:21-35: col_count = len(data), row_count = len(data[0]);
        copies data[i][j] for i < COLS, j < ROWS (panics if data is smaller)."""
        COLS = len(data) if COLS is None else COLS
        ROWS = len(data[0]) if ROWS is None else ROWS
        dt = _infer_dtype([x for col in data for x in col] or [0.0], dtype)
        temp = np.zeros((COLS, ROWS), dtype=dt)
        try:
            for i in range(COLS):
                for j in range(ROWS):
                    temp[i, j] = data[i][j]
        except IndexError as e:
            raise Panic(f"index out of bounds: {e}") from None
        return cls(ROWS, COLS, len(data), len(data[0]), temp)

    def get_col(self, col_index: int) -> np.ndarray:
        if not 0 <= col_index < self.COLS:
            raise Panic(f"index out of bounds: the len is {self.COLS} but the index is {col_index}")
        v = self.data[col_index].view()
        v.flags.writeable = False
        return v

    def get_col_mut(self, col_index: int) -> np.ndarray:
        if not 0 <= col_index < self.COLS:
            raise Panic(f"index out of bounds: the len is {self.COLS} but the index is {col_index}")
        return self.data[col_index]

    def get_dims(self) -> MatDim:
        return MatDim(rows=self.row_count, cols=self.col_count)

    def __eq__(self, other) -> bool:
        if not isinstance(other, DenseS):
            return NotImplemented
        return (
            (self.ROWS, self.COLS, self.col_count, self.row_count) == (other.ROWS, other.COLS, other.col_count, other.row_count)
            and bool(np.all(self.data == other.data))
        )

    def __repr__(self) -> str:
        return f"DenseS<{self.ROWS},{self.COLS}> {{ col_count: {self.col_count}, row_count: {self.row_count}, data: {self.data.tolist()} }}"
