"""sfl_amd/hostpipe.py's host-side pieces on the CPU (the GPU pipeline
itself: tests/test_gpu_party_pipeline.py)."""
import numpy as np
import pytest

from sfl_amd import hostpipe as H


@pytest.mark.parametrize("n", [1, 1023, 1 << 20, (1 << 20) + 1, 2_500_003, 100_000_000, 600_000_001])
def test_chunk_bounds_cover_and_align(n):
    b = H.chunk_bounds(n)
    assert b[0][0] == 0 and b[-1][1] == n
    assert all(hi0 == lo1 for (_, hi0), (lo1, _) in zip(b, b[1:]))
    assert all(lo % 1024 == 0 and lo < hi for lo, hi in b)
    assert all(hi - lo <= (1 << 24) for lo, hi in b)
    if n >= 8 << 20:
        assert len(b) >= 8
    assert H.chunk_bounds(0) == []


def test_fresh_output_chunks():
    n = 3_000_001
    b = H.chunk_bounds(n)
    f = H.FreshOutput(n, np.uint64, b)
    parts = [f.ready(j) for j in range(len(b))]
    assert sum(p.size for p in parts) == n and all(np.shares_memory(p, f.array) for p in parts)
    f.close()
    a = f.array
    assert a.shape == (n,) and a.dtype == np.uint64 and a.flags.writeable and a.flags.c_contiguous
    a[:] = 7
    assert int(a.sum()) == 7 * n


def test_host_layers_keep_contiguous_memory():
    x = np.arange(12, dtype=np.float32)
    y = np.arange(12, dtype=np.float32).reshape(3, 4).T
    got = H.host_layers([x, y, x.astype(np.float64)], np.float32)
    assert np.shares_memory(got[0], x)  # copied from in place
    assert not np.shares_memory(got[1], y) and np.array_equal(got[1], y.reshape(-1))
    assert got[2].dtype == np.float32


class _FakeHip:
    """hipHostRegister / Unregister stand-ins (no GPU here)."""

    def __init__(self):
        self.live = set()

    def hipHostRegister(self, p, n, f):
        self.live.add(p.value)
        return 0

    def hipHostUnregister(self, p):
        self.live.discard(p.value)
        return 0

    def hipGetLastError(self):
        return 0


def test_result_pool_recycles_only_dropped_buffers(monkeypatch):
    fake = _FakeHip()
    monkeypatch.setattr(H, "_hip", lambda: fake)
    pool = H.ResultPool(64 << 20)
    a = pool.take(16 << 20)
    assert a is not None and a.nbytes == 16 << 20 and len(fake.live) == 1
    view = a[:1024].view(np.uint64)[3:9]  # a derived view keeps its owner busy
    del a
    b = pool.take(16 << 20)
    assert b is not None and len(pool.bufs) == 2  # the first is still viewed
    del view
    c = pool.take(8 << 20)
    assert c is not None and len(pool.bufs) == 2 and c is pool.bufs[0]  # recycled, best fit
    assert pool.take(40 << 20) is None  # over the cap: the caller takes the fresh path
    assert pool.take(1 << 20) is None  # small results never pool
    del b, c
    pool.clear()
    assert pool.bufs == [] and fake.live == set()


def test_fresh_output_takes_a_pooled_buffer(monkeypatch):
    fake = _FakeHip()
    monkeypatch.setattr(H, "_hip", lambda: fake)
    monkeypatch.setattr(H, "RESULTS", H.ResultPool(64 << 20))
    n = 3_000_001
    f = H.FreshOutput(n, np.float64, H.chunk_bounds(n))
    assert f.stats["pooled"] and f.array.shape == (n,) and f.array.dtype == np.float64
    assert all(f.ready(j).size for j in range(len(f.bounds)))
    f.close()
    first = f.array.base
    del f
    g = H.FreshOutput(n, np.float64, H.chunk_bounds(n))
    assert g.stats["pooled"] and g.array.base is not first  # the first result is still alive (first holds it)
    del first
    keep = g.array
    del g
    h = H.FreshOutput(n - 5, np.uint64, H.chunk_bounds(n - 5))
    assert h.stats["pooled"] and not np.shares_memory(h.array, keep)
