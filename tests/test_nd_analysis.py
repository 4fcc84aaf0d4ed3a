"""The host analysis of solve(order="nd") (bsm_nd_analyse, csrc/nd_order.cpp):
no device use, so these run on the CPU.

Checked on 2-D Poisson grids, random sparse patterns and disconnected graphs:
the permutation, the post-order tree (levels = heights), the separator
property every front relies on (each edge lands inside one front), and the
front rows against a plain symbolic elimination of P A P^T."""
import numpy as np
import pytest
import scipy.sparse as sp

from basic_sparse_matrix_amd.solver import nd_analyse


def poisson_pattern(g):
    n = g * g
    idx = np.arange(n).reshape(g, g)
    rows, cols = [idx.ravel()], [idx.ravel()]
    for di, dj in ((0, 1), (1, 0)):
        a = idx[: g - di, : g - dj].ravel()
        b = idx[di:, dj:].ravel()
        rows += [a, b]
        cols += [b, a]
    m = sp.csr_matrix((np.ones(sum(len(r) for r in rows)), (np.concatenate(rows), np.concatenate(cols))), shape=(n, n))
    m.sum_duplicates()
    m.sort_indices()
    return m


def random_pattern(n, deg, seed):
    rng = np.random.default_rng(seed)
    r = rng.integers(0, n, n * deg)
    c = rng.integers(0, n, n * deg)
    m = sp.coo_matrix((np.ones(len(r)), (r, c)), shape=(n, n)).tocsr()
    m = m + m.T + sp.identity(n, format="csr")
    m.sum_duplicates()
    m.sort_indices()
    return m


def lower_only(m):
    lo = sp.tril(m).tocsr()
    lo.sort_indices()
    return lo


def edges(m):
    coo = sp.tril(m, k=-1).tocoo()
    return coo.row.astype(np.int64), coo.col.astype(np.int64)


def symbolic_columns(n, adj_lower_new):
    """L's column structures for the ordered graph: struct(j) = later
    neighbours of j, merged with struct(c) - {j} for every elimination-tree
    child c of j."""
    struct = [set() for _ in range(n)]
    kids = [[] for _ in range(n)]
    for j in range(n):
        s = set(adj_lower_new[j])
        for c in kids[j]:
            s |= struct[c]
        s.discard(j)
        struct[j] = s
        if s:
            kids[min(s)].append(j)
    return struct


def check_plan(m, leaf, exact_struct=True):
    n = m.shape[0]
    plan = nd_analyse(n, m.indptr, m.indices, leaf)
    perm = plan["perm"]
    assert np.array_equal(np.sort(perm), np.arange(n))
    pinv = np.empty(n, dtype=np.int64)
    pinv[perm] = np.arange(n)
    start, end, parent, level = plan["start"], plan["end"], plan["parent"], plan["level"]
    nn = len(start)
    # own columns tile [0, n) in post-order
    assert start[0] == 0 and end[-1] == n
    assert np.all(start[1:] == end[:-1]) and np.all(end >= start)
    owner = np.repeat(np.arange(nn), end - start)
    for i in range(nn):
        p = parent[i]
        if p >= 0:
            assert p > i and level[p] > level[i]
            assert plan["slot"][i] in (0, 1)
    assert parent[-1] == -1

    def ancestors(i):
        out = set()
        while parent[i] >= 0:
            i = parent[i]
            out.add(i)
        return out

    # every edge (a < b in the new order) lands in the front of a's node
    r, c = edges(m)
    a, b = np.minimum(pinv[r], pinv[c]), np.maximum(pinv[r], pinv[c])
    for x, y in zip(a.tolist(), b.tolist()):
        node = owner[x]
        if y >= end[node]:
            assert y in set(plan["st"][node].tolist())
    # front rows: ascending, past the node's columns, owned by ancestors
    for i in range(nn):
        s = plan["st"][i]
        assert np.all(np.diff(s) > 0)
        if len(s):
            assert s[0] >= end[i]
            anc = ancestors(i)
            assert set(owner[s].tolist()) <= anc
    if exact_struct:
        adj = [[] for _ in range(n)]
        for x, y in zip(a.tolist(), b.tolist()):
            adj[x].append(y)
        cols = symbolic_columns(n, adj)
        for i in range(nn):
            want = set()
            for j in range(start[i], end[i]):
                want |= {q for q in cols[j] if q >= end[i]}
            got = set(plan["st"][i].tolist())
            # a child subtree that touches no own column of the node still
            # passes its rows up through the node's front: a superset of L's
            # structure (extra explicit zeros), never a missing row
            assert want <= got, i
            kid_rows = set()
            for k in np.nonzero(parent == i)[0]:
                kid_rows |= {q for q in plan["st"][k].tolist() if q >= end[i]}
            assert got == want | kid_rows, i
    return plan


@pytest.mark.parametrize("g,leaf", [(1, 256), (2, 1), (5, 4), (12, 8), (20, 16), (31, 64)])
def test_poisson_grids(g, leaf):
    m = poisson_pattern(g)
    plan = check_plan(m, leaf)
    # a 2-D grid bisects: separators much smaller than the grid side squared
    if g * g > 4 * leaf:
        assert plan["level"].max() >= 2
        root = len(plan["start"]) - 1
        assert plan["end"][root] - plan["start"][root] <= 2 * g


def test_lower_triangle_only_gives_the_same_plan():
    m = poisson_pattern(15)
    full = nd_analyse(m.shape[0], m.indptr, m.indices, 16)
    lo = lower_only(m)
    low = nd_analyse(lo.shape[0], lo.indptr, lo.indices, 16)
    assert np.array_equal(full["perm"], low["perm"])


@pytest.mark.parametrize("n,deg,seed,leaf", [(50, 2, 0, 8), (300, 1, 1, 16), (400, 3, 2, 32)])
def test_random_patterns(n, deg, seed, leaf):
    check_plan(random_pattern(n, deg, seed), leaf)


def test_disconnected():
    # diagonal matrix (no edges) and two grids side by side
    d = sp.identity(500, format="csr")
    check_plan(d, 16)
    g = poisson_pattern(10)
    m = sp.block_diag([g, g, sp.identity(7)], format="csr")
    m.sort_indices()
    check_plan(m, 8)


def test_unsorted_row_is_refused():
    import ctypes

    from basic_sparse_matrix_amd import _lib

    rp = np.array([0, 2, 4], dtype=np.uint64)
    ci = np.array([1, 0, 0, 1], dtype=np.uint64)  # row 0 unsorted
    nn, sl = ctypes.c_uint64(0), ctypes.c_uint64(0)
    rc = _lib.load().bsm_nd_analyse(2, _lib.ptr(rp), _lib.ptr(ci), 4, None, None, 0, ctypes.byref(nn), None, 0,
                                    ctypes.byref(sl))
    assert rc == 7  # BSM_ERR_UNSUPPORTED
