"""Host-side panics of the mirror that need no device (CPU): the reference's
loop order decides WHICH out-of-range read panics first."""

import numpy as np
import pytest

from basic_sparse_matrix_amd import Csr, DenseS, Panic


def short_rhs(len0, len1, rows=4):
    class Short(DenseS):  # DenseS with ROWS > len(col): get_col(c) is shorter than ROWS
        ROWS = rows
        COLS = 2

        def __init__(self):
            self.data = [np.ones(len0), np.ones(len1)]

        def get_col(self, j):
            return self.data[j]

        def get_dims(self):
            from basic_sparse_matrix_amd.util import MatDim

            return MatDim(rows=rows, cols=2)

    return Short()


def test_short_column_panics_at_first_read_in_reference_order():
    # row 0: cols [1, 3]; row 1: cols [2]; row 2: [0, 3]
    a = Csr.from_csr_arrays((3, 4), np.array([0, 2, 3, 5], np.uint64), np.array([1, 3, 2, 0, 3], np.uint64),
                            np.ones(5))
    # column 0 has length 3 (index 3 is out of range), column 1 length 2 (2, 3 out of range).
    # Row 0, c = 0: entries (1 ok, 3 BAD) -> the panic names index 3 with len 3
    with pytest.raises(Panic, match="the len is 3 but the index is 3"):
        a.mul_dense_s(short_rhs(3, 2))
    # column 0 long enough: row 0, c = 1: entry col 1 ok, col 3 bad (len 2) -> index 3, len 2
    with pytest.raises(Panic, match="the len is 2 but the index is 3"):
        a.mul_dense_s(short_rhs(4, 2))
    # only column 1 short at len 3: first bad in row order is row 0's col 3
    with pytest.raises(Panic, match="the len is 3 but the index is 3"):
        a.mul_dense_s(short_rhs(4, 3))
