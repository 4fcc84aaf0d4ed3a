"""Shared types of the reference crate (src/util.rs): MatDim, GetDims, MatErr.

Rust ``Result<_, MatErr>`` maps to raising :class:`MatErr` (with ``.kind``);
a Rust ``panic!`` (index out of bounds, ``unwrap`` on ``None``, "big eek")
maps to raising :class:`Panic`.
"""

from __future__ import annotations

import enum
from dataclasses import dataclass


@dataclass(frozen=True)
class MatDim:
    """util.rs:11-33. ``MatDim.from_tuple((rows, cols))`` mirrors
    ``From<(usize,usize)>`` (util.rs:23-27): rows first."""

    rows: int
    cols: int

    def transpose(self) -> "MatDim":
        return MatDim(self.cols, self.rows)

    @staticmethod
    def of(d) -> "MatDim":
        if isinstance(d, MatDim):
            return d
        rows, cols = d
        return MatDim(int(rows), int(cols))

    def as_tuple(self):
        return (self.rows, self.cols)

    def __str__(self) -> str:  # util.rs:29-33
        return f"(rows: {self.rows}, cols: {self.cols})"


class MatErrKind(enum.Enum):
    """util.rs:47-55."""

    MatrixFinalised = "MatrixFinalised"
    MatrixNotFinalised = "MatrixNotFinalised"
    NonSquareMatrix = "NonSquareMatrix"
    IncorrectDimensions = "IncorrectDimensions"
    PaddingSizeSmallerThanOriginal = "PaddingSizeSmallerThanOriginal"
    OutOfBounds = "OutOfBounds"


class MatErr(Exception):
    """``Err(MatErr::<kind>)``. Compares equal to another MatErr of the same kind."""

    def __init__(self, kind: MatErrKind):
        super().__init__(kind.value)
        self.kind = kind

    def __eq__(self, other):
        return isinstance(other, MatErr) and other.kind == self.kind

    def __hash__(self):
        return hash(self.kind)


class Panic(RuntimeError):
    """The reference would ``panic!`` on this input."""


class GetDims:
    """util.rs:43-45."""

    def get_dims(self) -> MatDim:  # pragma: no cover - interface
        raise NotImplementedError
