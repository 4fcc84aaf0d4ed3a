"""The Python host mirror of the reference API (basic_sparse_matrix_amd/sparse.py)
against the reference's own #[test] vectors (tests/golden/reference_unit_tests.json):
construction (from_data, insert_unchecked, create_diagonal), the row accessors
get_row_compact / get_row_complete (src/sparse.rs:252-294), the entry iterator
and the CSR arrays. Host-only: no device is touched."""

import numpy as np
import pytest

from basic_sparse_matrix_amd import Csr

DT = {"i32": np.int32, "f32": np.float32, "f64": np.float64, "u32": np.uint32}


def _csr(rows, dtype):
    return Csr.from_data([list(r) for r in rows], dtype=DT[dtype])


@pytest.mark.parametrize("name", ["example_mat_0", "example_mat_1", "example_mat_2",
                                  "csr_with_empty_row_top", "csr_with_empty_row_middle"])
def test_from_data_arrays(golden, name):
    g = golden[name]
    m = _csr(g["rows"], g["dtype"])
    assert [int(x) for x in m.v] == g["v"]
    assert [int(x) for x in m.col_index] == g["col_index"]
    assert [int(x) for x in m.row_index] == g["row_index"]


def test_get_row_by_index_0(golden):
    g = golden["get_row_by_index_0"]
    m = _csr(g["rows"], g["dtype"])
    assert [int(x) for x in m.get_row_complete(g["row"])] == g["complete"]
    got = [[int(e.v), e.row_index, e.col_index] for e in m.get_row_compact(g["row"])]
    assert got == g["compact"]


def test_get_row_by_index_1(golden):
    g = golden["get_row_by_index_1"]
    m = _csr(g["rows"], g["dtype"])
    for r, (complete, compact) in enumerate(zip(g["complete"], g["compact"])):
        assert [int(x) for x in m.get_row_complete(r)] == complete
        assert [[int(e.v), e.row_index, e.col_index] for e in m.get_row_compact(r)] == compact
    # past the last row: None (sparse.rs:270)
    assert m.get_row_complete(len(g["rows"]) + 1) is None


def test_get_row_by_index_single(golden):
    """insert_unchecked into an unfinalised 5x5 f32 matrix: the last recorded
    row extends to v.len() (sparse.rs:256-260, 274-278)."""
    g = golden["get_row_by_index_single"]
    m = Csr.new(tuple(g["dims"]), dtype=DT[g["dtype"]])
    for val, r, c in g["insert_unchecked"]:
        m._insert_unchecked(DT[g["dtype"]](float(val)), r, c)
    row = m.get_row_complete(g["row"])
    assert row[0] == DT[g["dtype"]](float(g["complete0"]))
    assert len(row) == g["dims"][1]


def test_iterator(golden):
    g = golden["test_iterator"]
    m = _csr(g["rows"], g["dtype"])
    got = [[int(e.v), e.row_index, e.col_index] for e in m]
    assert got == g["entries"]


def test_create_diagonal(golden):
    g = golden["create_diagonal"]
    for case in g["cases"]:
        m = Csr.create_diagonal(case["diag"], dtype=DT[g["dtype"]])
        n = len(case["diag"])
        dense = [[int(x) for x in m.get_row_complete(r)] for r in range(n)]
        assert dense == case["rows"]
