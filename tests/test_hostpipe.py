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


def test_fresh_output_pages_and_chunks():
    n = 3_000_001
    b = H.chunk_bounds(n)
    f = H.FreshOutput(n, np.uint64, b)
    assert f.base % H.PAGE == 0  # page-aligned: every chunk registers its own pages
    spans = [f._span(lo, hi) for lo, hi in b]
    assert all(s0 % H.PAGE == 0 and s1 % H.PAGE == 0 for s0, s1 in spans)
    assert all(a[1] <= c[0] for a, c in zip(spans, spans[1:]))  # no page in two chunks
    for fs in f._futs:
        for x in fs:
            x.result()
    a = f.array
    assert a.shape == (n,) and a.dtype == np.uint64 and a.flags.writeable
    a[:] = 7
    assert int(a.sum()) == 7 * n
    f.registered = []  # nothing registered on the CPU
    f.close()
    del f
    assert int(a[-1]) == 7  # the caller's array keeps the mapping alive


def test_host_layers_keep_contiguous_memory():
    x = np.arange(12, dtype=np.float32)
    y = np.arange(12, dtype=np.float32).reshape(3, 4).T
    got = H.host_layers([x, y, x.astype(np.float64)], np.float32)
    assert np.shares_memory(got[0], x)  # registered in place
    assert not np.shares_memory(got[1], y) and np.array_equal(got[1], y.reshape(-1))
    assert got[2].dtype == np.float32
