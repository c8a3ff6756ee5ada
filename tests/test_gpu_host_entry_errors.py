"""Error paths of the blocking host-array entries (include/sfl_sa.h:
sa_fused_clients_host_f32, sa_clients_host, sa_mask_host,
sa_sum_decode_host).

Each entry enqueues its host-to-device copy before the launch function that
validates ``fxp_bits`` runs, so a call with ``fxp_bits = 63`` fails AFTER
work that reads the caller's pinned scratch is on the stream.  The contract
(sa_api.hip, the comment above ``drain``): an error returned after the first
copy was enqueued leaves the stream drained, so the caller may reuse or free
the scratch at once.  Checked here directly -- the stream is idle the moment
the failing call returns -- and functionally: the pinned scratch is
scribbled over right away and the very same scratch then serves a good call
whose outputs must be bit-exact against the oracle.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import secagg as o  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"
N = 2_000_003  # ~8-16 MB per copy: a copy still in flight at return would be seen by query()


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd import _lib as L

    L.lib()


def _inputs(c, n=N, dtype=np.float32):
    rng = np.random.default_rng(1000 + c)
    x = rng.standard_normal(n) * 3
    return x.astype(np.int64) if dtype == np.int64 else x.astype(dtype)


def _scratch(pin_bytes, dev_bytes):
    pinned = torch.empty(pin_bytes, dtype=torch.uint8).pin_memory()
    dev = torch.empty(dev_bytes, dtype=torch.uint8, device=DEV)
    return pinned, dev


def _streams_for(c, names, offset=0):
    """client c's streams in its masker's order (peers by index), oracle seeds"""
    from sfl_amd import _lib as L

    out = []
    for j in range(len(names)):
        if j == c:
            continue
        seed = o.pair_seed(min(c, j), max(c, j))
        out.append((L.pcg64_advance(L.pcg64_from_seed(seed), offset), 1 if j > c else -1, j))
    return out


def _oracle_masked(x, c, names, offset=0, weight=None):
    q = o.quantize(x, weight)
    seeds = {names[j]: o.pair_seed(min(c, j), max(c, j)) for j in range(len(names)) if j != c}
    return o.mask_client(q, names[c], seeds, offset)


def _fail_then_idle(call):
    from sfl_amd import _lib as L

    torch.cuda.synchronize()
    with pytest.raises(L.SALibraryError, match="code -1"):
        call()
    # drained on return: nothing of the failed call is still reading the scratch
    assert torch.cuda.current_stream(DEV).query()


def test_mask_host_error_after_copy_drains_then_reuse_is_exact():
    from sfl_amd import kernels as K

    names = ["a", "b", "c"]
    x = _inputs(0)
    pinned, dev = _scratch(*K.mask_host_scratch(N, 4))
    st = _streams_for(0, names, offset=12345)
    _fail_then_idle(lambda: K.mask_host(x, np.float32, st, pinned, dev, fxp_bits=63))
    pinned.fill_(0xA5)
    dev.fill_(0x5A)
    out, flags = K.mask_host(x, np.float32, st, pinned, dev)
    assert flags == 0
    assert np.array_equal(out, _oracle_masked(x, 0, names, offset=12345))


def test_sum_decode_host_error_after_copy_drains_then_reuse_is_exact():
    from sfl_amd import kernels as K

    names = ["a", "b", "c"]
    masked = [_oracle_masked(_inputs(c), c, names) for c in range(3)]
    pinned, dev = _scratch(*K.sum_decode_host_scratch(3, N))
    _fail_then_idle(lambda: K.sum_decode_host(masked, pinned, dev, fxp_bits=63))
    pinned.fill_(0xA5)
    out, dig = K.sum_decode_host(masked, pinned, dev, divisor=3.0)
    s = o.server_sum(masked)
    assert np.array_equal(out, o.decode(s, divisor=3.0))
    assert [int(d) for d in dig] == [o.digest(m) for m in masked]


@pytest.mark.parametrize("dtype", [np.float64, np.int64])
def test_clients_host_error_after_copy_drains_then_reuse_is_exact(dtype):
    from sfl_amd import kernels as K

    names = ["a", "b", "c", "d"]
    xs = [_inputs(c, dtype=dtype) for c in range(4)]
    streams = [_streams_for(c, names) for c in range(4)]
    w = [1.0] * 4
    pinned, dev = _scratch(*K.host_clients_scratch(4, N, 8))
    _fail_then_idle(lambda: K.clients_host(xs, dtype, w, streams, pinned, dev, fxp_bits=63))
    pinned.fill_(0xA5)
    dev.fill_(0x5A)  # the large-sum branch fills its sum on the device: stale bytes must not leak in
    out, dig, flags = K.clients_host(xs, dtype, w, streams, pinned, dev, divisor=4.0)
    masked = [_oracle_masked(xs[c], c, names) for c in range(4)]
    assert flags == 0
    assert [int(d) for d in dig] == [o.digest(m) for m in masked]
    assert np.array_equal(out, o.decode(o.server_sum(masked), divisor=4.0))


def test_fused_clients_host_f32_error_after_copy_drains_then_reuse_is_exact():
    from sfl_amd import _lib as L
    from sfl_amd import kernels as K

    C = 4
    names = [f"p{c}" for c in range(C)]
    xs = [_inputs(c) for c in range(C)]
    gens, signs = [], []
    for u in range(C):
        for v in range(u + 1, C):
            gens.append(L.pcg64_from_seed(o.pair_seed(u, v)))
            signs.append(1)
    pinned, dev = _scratch(*K.host_fused_scratch(C, N))
    _fail_then_idle(lambda: K.fused_clients_host_f32(xs, [1.0] * C, gens, signs, pinned, dev, fxp_bits=63))
    pinned.fill_(0xA5)
    dev.fill_(0x5A)
    res = K.fused_clients_host_f32(xs, [1.0] * C, gens, signs, pinned, dev, divisor=float(C))
    assert res is not None
    out, dig, flags = res
    masked = [_oracle_masked(xs[c], c, names) for c in range(C)]
    assert flags == 0
    assert [int(d) for d in dig] == [o.digest(m) for m in masked]
    assert np.array_equal(out, o.decode(o.server_sum(masked), divisor=float(C)))
