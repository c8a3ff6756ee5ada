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


def test_pcopy_and_pieces():
    src = np.arange(11_000_003, dtype=np.float64)
    dst = np.empty_like(src)
    H.pcopy(dst, src)  # several 4 MiB+ pieces on the pool
    assert np.array_equal(dst, src)
    small = np.arange(10, dtype=np.int64)
    d2 = np.zeros_like(small)
    H.pcopy(d2, small)
    assert np.array_equal(d2, small)
    layers = [np.arange(5), np.zeros(0, np.int64), np.arange(100, 107), np.arange(200, 203)]
    flat = np.concatenate(layers)
    for lo, hi in [(0, 15), (3, 9), (5, 12), (12, 15), (4, 5)]:
        got = np.full(hi - lo, -1)
        for a, off in H.pieces(layers, lo, hi):
            got[off:off + a.size] = a
        assert np.array_equal(got, flat[lo:hi]), (lo, hi)


def test_host_layers_keep_contiguous_memory():
    x = np.arange(12, dtype=np.float32)
    y = np.arange(12, dtype=np.float32).reshape(3, 4).T
    got = H.host_layers([x, y, x.astype(np.float64)], np.float32)
    assert np.shares_memory(got[0], x)  # staged from in place
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


def test_pinned_takes_pooled_arrays_as_they_are(monkeypatch):
    fake = _FakeHip()
    monkeypatch.setattr(H, "_hip", lambda: fake)
    monkeypatch.setattr(H, "RESULTS", H.ResultPool(64 << 20))
    pooled = H.RESULTS.take(16 << 20)[: 8 << 20].view(np.uint64)
    other = np.ones(1 << 20, np.uint64)
    assert H.RESULTS.contains(pooled[10:20]) and not H.RESULTS.contains(other)
    before = set(fake.live)
    with H.Pinned([pooled], register=False) as p:
        assert p.ok and fake.live == before  # nothing new registered
    with H.Pinned([pooled, other], register=False) as p:
        assert not p.ok  # the caller stages instead
    with H.Pinned([pooled, other]) as p:
        assert p.ok and len(fake.live) == len(before) + 1
    assert fake.live == before
