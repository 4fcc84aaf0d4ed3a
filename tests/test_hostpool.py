"""Host result pool (basic_sparse_matrix_amd/hostpool.py): recycled mappings
must never be handed out while any array made from them is alive."""
import gc

import numpy as np

from basic_sparse_matrix_amd import hostpool


def _addr(a):
    return a.__array_interface__["data"][0]


def test_pool_reuses_a_dropped_mapping_and_aligns_it():
    p = hostpool.HostPool(1 << 30)
    a = p.empty(3_000_000, np.uint64)
    assert a.shape == (3_000_000,) and a.dtype == np.uint64
    assert _addr(a) % (2 << 20) == 0
    a[:] = 7
    addr = _addr(a)
    del a
    gc.collect()
    assert p.free_bytes > 0
    b = p.empty(3_000_000, np.float64)
    assert _addr(b) == addr and p.hits == 1


def test_live_slice_keeps_the_mapping_out_of_the_pool():
    p = hostpool.HostPool(1 << 30)
    a = p.empty(2_000_000, np.float64)
    a[:] = np.arange(a.size)
    s = a[10:20]
    del a
    gc.collect()
    assert p.free_bytes == 0  # the slice still uses it
    b = p.empty(2_000_000, np.float64)
    b[:] = -1
    assert np.array_equal(s, np.arange(10, 20, dtype=np.float64))
    assert _addr(b) != _addr(s) - 80
    del s
    gc.collect()
    assert p.free_bytes > 0


def test_size_classes_and_cap():
    p = hostpool.HostPool(8 << 20)  # keeps at most 8 MiB free
    a = p.empty(1 << 20, np.uint64)  # 8 MiB
    b = p.empty(1 << 20, np.uint64)
    del a, b
    gc.collect()
    assert p.free_bytes <= 8 << 20
    big = p.empty(4 << 20, np.uint64)  # 32 MiB: no free mapping is close enough
    assert big.size == 4 << 20 and p.hits == 0
    small = p.empty(1 << 20, np.uint64)
    assert p.hits == 1 and small.size == 1 << 20


def test_module_empty_small_and_disabled(monkeypatch):
    small = hostpool.empty(100, np.int32)
    assert small.shape == (100,) and small.base is None  # plain numpy below the threshold
    monkeypatch.setenv("BSM_HOST_POOL", "0")
    big = hostpool.empty(4 << 20, np.float64)
    assert big.base is None and big.size == 4 << 20


def test_give_back_during_take_scan_keeps_the_chosen_mapping():
    """a give-back (a finalizer run by GC on the same thread) while
    _take scans the free list must not make it remove a different mapping."""
    H = 2 << 20
    p = hostpool.HostPool(64 * H)
    small, big = hostpool._Mapping(2 * H), hostpool._Mapping(4 * H)
    p._give_back(small)
    p._give_back(big)
    late = hostpool._Mapping(2 * H)

    class Hooked(list):
        fired = False

        def __iter__(self):
            it = super().__iter__()
            for m in it:
                if not Hooked.fired:
                    Hooked.fired = True
                    p._give_back(late)  # lands while the scan runs
                yield m

    p._free = Hooked(p._free)
    got = p._take(4 * H)  # only `big` fits (small is too small, late arrives mid-scan)
    assert got is big
    assert any(m is small for m in p._free) and any(m is late for m in p._free)
    assert not any(m is big for m in p._free)
    assert p.free_bytes == 4 * H
