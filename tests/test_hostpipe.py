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


class _RangeHip(_FakeHip):
    """Records every registration's range; refuses every one after the
    first ``allow`` (the driver turning memory down mid-call)."""

    def __init__(self, allow=None):
        super().__init__()
        self.ranges, self.allow = [], allow

    def hipHostRegister(self, p, n, f):
        if self.allow is not None and len(self.ranges) >= self.allow:
            return 1
        self.ranges.append((p.value, p.value + n.value))
        return super().hipHostRegister(p, n, f)


def _parties(C, n, dtype=np.float32, shift=0):
    """C parties' one-layer payloads whose data start ``shift`` bytes into a
    page plus numpy's own offset (the same for all: one allocator)."""
    out = []
    for _ in range(C):
        raw = np.empty(n * np.dtype(dtype).itemsize + 2 * H.PAGE, np.uint8)
        a0 = -raw.ctypes.data % H.PAGE + 16 + shift
        out.append([raw[a0:a0 + n * np.dtype(dtype).itemsize].view(dtype)])
    return out


@pytest.mark.parametrize("dtype", [np.float32, np.float64, np.int64])
def test_page_bounds_put_joins_on_pages(dtype):
    n = 20_000_003
    ll = _parties(3, n, dtype)
    b = H.page_bounds(H.chunk_bounds(n), ll)
    assert b[0][0] == 0 and b[-1][1] == n and len(b) == len(H.chunk_bounds(n))
    assert all(hi0 == lo1 for (_, hi0), (lo1, _) in zip(b, b[1:]))
    for lo, _ in b[1:]:
        assert lo * np.dtype(dtype).itemsize % 16 == 0
        assert all((p[0].ctypes.data + lo * p[0].itemsize) % H.PAGE == 0 for p in ll), lo
    # parties at different page offsets: no common join, the bounds stay
    mixed = _parties(2, n, dtype) + _parties(1, n, dtype, shift=32)
    assert H.page_bounds(H.chunk_bounds(n), mixed) == H.chunk_bounds(n)
    # a join inside a later layer moves inside that layer, unless the page
    # boundary there is not 16-byte aligned in elements (device slices)
    for first in (3_000_001, 3_000_004):
        two = [[(np.zeros(first, dtype)), _parties(1, n, dtype)[0][0]]]
        base = H.chunk_bounds(n + first)
        b2 = H.page_bounds(base, two)
        moved = 0
        for (lo, _), (lo0, _) in zip(b2[1:], base[1:]):
            li = 1 if lo >= first else 0
            on_page = (two[0][li].ctypes.data + (lo - (first if li else 0)) * two[0][li].itemsize) % H.PAGE == 0
            assert on_page or lo == lo0, lo
            assert lo * np.dtype(dtype).itemsize % 16 == 0
            moved += li == 1 and on_page
        if first % 4 == 0:  # every join inside the second layer lands on a page
            assert moved == sum(lo0 >= first for lo0, _ in base[1:])


def _split_all(pin, layers, bounds):
    """Every chunk's pieces through ``split``: (piece, ranges) in order."""
    out = []
    for lo, hi in bounds:
        for a, _ in H.pieces(layers, lo, hi):
            out.append((a, pin.split(a)))
    return out


def test_lazy_pinned_registers_chunk_by_chunk(monkeypatch):
    fake = _RangeHip()
    monkeypatch.setattr(H, "_hip", lambda: fake)
    monkeypatch.setattr(H, "LAZY_GROWTH", 1)
    n = 40_000_000  # 160 MB: lazily registered
    ll = _parties(2, n)
    bounds = H.page_bounds(H.chunk_bounds(n), ll)
    arrays = [a for p in ll for a in p]
    with H.Pinned(arrays, lazy=True) as pin:
        assert pin.ok and fake.ranges == []  # nothing registered on entry
        got = _split_all(pin, ll[0], bounds)
        # joins on pages: every piece is one registered range
        assert all(r == [(0, a.nbytes, True)] for a, r in got)
        p0 = arrays[0].ctypes.data
        mine = sorted(r for r in fake.ranges if p0 - H.PAGE < r[0] < p0 + n * 4)
        assert all(r0 % H.PAGE == 0 and r1 % H.PAGE == 0 for r0, r1 in mine)
        assert all(a1 == b0 for (_, a1), (b0, _) in zip(mine, mine[1:]))  # contiguous, no overlap
        assert mine[0][0] <= p0 and mine[-1][1] >= p0 + n * 4
        assert len(mine) == len(bounds)
        assert pin.stats["registrations"] == len(fake.ranges) and pin.stats["staged_bytes"] == 0
    assert fake.live == set()


def test_lazy_pinned_grows_geometrically(monkeypatch):
    """The default growth: chunk 0, then 1, then 2-3, 4-7, ... -- log2 of the
    chunk count registrations an array, copies cut only where a
    registration ends inside a chunk."""
    fake = _RangeHip()
    monkeypatch.setattr(H, "_hip", lambda: fake)
    monkeypatch.setattr(H, "LAZY_GROWTH", 2)
    n = 256_000_000
    ll = _parties(1, n)
    bounds = H.page_bounds(H.chunk_bounds(n, target=16), ll)
    assert len(bounds) == 16
    with H.Pinned(ll[0], lazy=True) as pin:
        got = _split_all(pin, ll[0], bounds)
        assert len(fake.ranges) == 5
        assert all(reg for _, r in got for _, _, reg in r)
        assert sum(len(r) - 1 for _, r in got) <= 4  # a sliver where a registration ends mid-chunk
        p0 = ll[0][0].ctypes.data
        for a, r in got:
            for b0, b1, _ in r:
                assert not any(a.ctypes.data + b0 < j < a.ctypes.data + b1 for j, _ in fake.ranges)
        assert fake.ranges[0][0] <= p0 and fake.ranges[-1][1] >= p0 + 4 * n


def test_lazy_pinned_cuts_copies_at_registration_joins(monkeypatch):
    fake = _RangeHip()
    monkeypatch.setattr(H, "_hip", lambda: fake)
    monkeypatch.setattr(H, "LAZY_GROWTH", 1)
    n = 20_000_003
    ll = [_parties(1, n, np.float64)[0]]
    bounds = H.chunk_bounds(n)  # joins off the pages: pieces straddle a join
    with H.Pinned(ll[0], lazy=True) as pin:
        got = _split_all(pin, ll[0], bounds)
        joins = {r0 for r0, _ in fake.ranges[1:]}
        for a, r in got:
            assert r[0][0] == 0 and r[-1][1] == a.nbytes and all(x[1] == y[0] for x, y in zip(r, r[1:]))
            assert all(reg for _, _, reg in r)
            for b0, b1, _ in r:  # no range contains a join inside it
                p0 = a.ctypes.data
                assert not any(p0 + b0 < j < p0 + b1 for j in joins)
        assert any(len(r) == 2 for _, r in got)


def test_lazy_pinned_refused_mid_call_stages_the_rest(monkeypatch):
    fake = _RangeHip(allow=3)  # 3 chunks, then refused
    monkeypatch.setattr(H, "_hip", lambda: fake)
    monkeypatch.setattr(H, "LAZY_GROWTH", 1)
    n = 40_000_000
    ll = _parties(1, n)
    bounds = H.page_bounds(H.chunk_bounds(n), ll)
    with H.Pinned(ll[0], lazy=True) as pin:
        got = _split_all(pin, ll[0], bounds)
        regs = [all(reg for _, _, reg in r) for _, r in got]
        assert regs[:3] == [True] * 3 and not any(regs[3:])
        assert pin.stats["staged_bytes"] == sum(a.nbytes for a, _ in got[3:])
    assert fake.live == set()
    # an array registered whole on entry and refused: nothing stays
    # registered, the caller stages (Feeder)
    fake = _RangeHip(allow=0)
    monkeypatch.setattr(H, "_hip", lambda: fake)
    with H.Pinned([np.ones(1 << 20, np.float32)], lazy=True) as pin:
        assert not pin.ok
