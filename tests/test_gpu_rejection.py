"""numpy's rejection re-draw, reproduced (VERDICT r1 "missing 3").

The reference's masks are ``Generator.integers(int64.min, int64.max)`` draws:
numpy's Lemire bounded draw REJECTS a raw PCG64 output of 0 and takes the
next raw output, so the stream runs one raw draw further along from that
element on (p = 2^-64 per draw).  A PCG64 state whose draw k is 0 is built
by walking back from a state with hi == lo (XSL-RR output 0).  The oracle is
numpy itself: persistent ``np.random.Generator`` objects per (party, peer)
(``oracle.secagg.OracleMaskers``), whose ``integers`` does the rejection.

GPU: masked vectors, digests, sums and decoded results of the plugin equal
the oracle's bit for bit in the round that hits the zero AND in the next
round (stream positions), on the fused, fused + wire-image, per-party wire
and host-fused paths.  CPU: the (element, shift) bookkeeping of
``kernels.rejected_draws`` for several rejections in one window.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import secagg as o  # noqa: E402

A = o.PCG64_MULT
M = (1 << 128) - 1


def forced_zero_state(k: int, inc: int = (12345 << 1) | 1, tag: int = 0xDEADBEEF) -> tuple:
    """(state, inc) whose raw draw k (0-based) is 0."""
    ainv = pow(A, -1, 1 << 128)
    s = (((tag << 64) | tag) - inc) * ainv & M  # state before the zero draw
    for _ in range(k):
        s = ((s - inc) * ainv) & M
    assert o.pcg64_raw_py(s, inc, k + 1)[k] == 0
    return s, inc


def test_rejected_draws_bookkeeping(monkeypatch):
    """Zeros at raw indices 5 and 9 (and 10) of a stream: element 5 moves to
    raw 6 (shift 1); raw 9 is then element 8 -> shift 2; raw 10 = element 8
    again -> shift 3; n + 3 raw draws consumed."""
    from sfl_amd import kernels as K

    zeros = {5, 9, 10}

    def adv(gen, d):
        return gen + d

    def find(gens, n, device):
        start = gens[0]
        for i in range(n):
            if start + i in zeros:
                return [i]
        return [None]

    monkeypatch.setattr(K.L, "pcg64_advance", adv)
    monkeypatch.setattr(K, "find_zero_draws", find)
    pts, total = K.rejected_draws(0, 20, None)
    assert pts == [(5, 1), (8, 2), (8, 3)]
    assert total == 23
    # element e uses raw e + shift(e): 0..4 -> 0..4, 5..7 -> 6..8, 8.. -> 11..
    used = []
    for e in range(20):
        sh = max([s for k, s in pts if k <= e], default=0)
        used.append(e + sh)
    assert not zeros & set(used) and used == sorted(set(used))
    pts, total = K.rejected_draws(0, 5, None)  # the zero lies beyond the window
    assert pts == [] and total == 5


def test_rejected_draws_many_searches_all_streams_at_once(monkeypatch):
    """The careful replay's search: one batched find over every stream, then
    only the streams with a hit are followed; the bookkeeping equals
    rejected_draws stream by stream."""
    from sfl_amd import kernels as K

    zeros = {5, 9, 10, 1005, 2000}
    calls = []

    def adv(gen, d):
        return gen + d

    def find(gens, n, device):
        calls.append(len(gens))
        out = []
        for start in gens:
            out.append(next((i for i in range(n) if start + i in zeros), None))
        return out

    monkeypatch.setattr(K.L, "pcg64_advance", adv)
    monkeypatch.setattr(K, "find_zero_draws", find)
    gens = [0, 100, 1000, 1990, 3000]
    got = K.rejected_draws_many(gens, 20, None)
    assert calls[0] == len(gens)  # one search over all of them first
    assert sum(1 for c in calls[1:] if c != 1) == 0  # then per-stream follow-ups only
    calls.clear()
    assert got == [K.rejected_draws(g, 20, None) for g in gens]
    assert [t for _, t in got] == [23, 20, 21, 21, 20]


def test_oracle_generator_rejects_zero():
    s, inc = forced_zero_state(5)
    raw = o.pcg64_raw_py(s, inc, 12)
    got = o.generator_from_state(s, inc).integers(o.INT64_MIN, o.INT64_MAX, size=10).astype(np.uint64)
    exp = [(r + o.MASK_OFFSET) & o.U64 for r in raw if r][:10]
    assert got.tolist() == exp


# --------------------------------------------------------------------- GPU
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd import _lib as L

    L.lib()


@pytest.mark.gpu
@pytest.mark.parametrize("k", [0, 5, 1027, 4097])
def test_find_zero_and_shift_match_numpy(k):
    _gpu()
    from sfl_amd import _lib as L
    from sfl_amd import kernels as K

    n = 5000
    s, inc = forced_zero_state(k)
    g = L.PCG64.of(s, inc)
    assert K.find_zero_draws([g, L.pcg64_from_seed(7)], n, "cuda:0") == [k, None]
    pts, total = K.rejected_draws(g, n, "cuda:0")
    assert pts == [(k, 1)] and total == n + 1
    # a masked vector built from the unshifted stream, moved onto numpy's
    out = torch.empty(n, dtype=torch.int64, device="cuda:0")
    x = torch.randn(n, device="cuda:0") * 1e-2
    flags = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    K.mask(x, out, [(g, -1, 0)], flags=flags)
    torch.cuda.synchronize()
    assert int(flags.item()) & L.SA_FLAG_PRG_REJECT
    K.stream_shift(out, g, -1, k, 1)
    dig = torch.zeros(1, dtype=torch.int64, device="cuda:0")
    K.xor_digest(out, dig)
    m = o.generator_from_state(s, inc).integers(o.INT64_MIN, o.INT64_MAX, size=n).astype(np.uint64)
    exp = o.quantize(x.cpu().numpy()) - m
    assert np.array_equal(K.as_u64(out), exp)
    assert int(K.as_u64(dig)[0]) == o.digest(exp)


NAMES = ["alice", "bob", "carol", "dave"]


def _pair_states(zero_pair, k):
    seeds = o.seeds_for(NAMES)
    st = {(a, b): seeds[a][b] for a in NAMES for b in NAMES if a < b}
    st[zero_pair] = forced_zero_state(k)
    return st


@pytest.mark.gpu
@pytest.mark.parametrize("mode", ["fused", "fused_images", "wire", "host_fused"])
def test_plugin_round_with_rejection_matches_numpy(mode):
    """The (bob, dave) pair stream draws a raw 0 at element 1000 of round 0:
    results, wire images, digests and the next round all equal numpy's."""
    _gpu()
    from sfl_amd.device import PYU, reveal
    from sfl_amd.security.aggregation import SecureAggregator

    n = 3001
    pair = _pair_states(("bob", "dave"), 1000)
    pyus = [PYU(nm, 0) for nm in NAMES]
    fused = mode != "wire"
    keep = mode in ("fused_images", "wire")
    agg = SecureAggregator(PYU("server", 0), pyus, seeds=pair, fused=fused, keep_masked=keep)
    ora = o.OracleMaskers(NAMES, pair)
    rng = np.random.default_rng(11)
    for rnd in range(2):
        xs = [(rng.standard_normal(n) * 1e-2).astype(np.float32) for _ in NAMES]
        if mode == "host_fused":
            objs = [p(lambda x=x: x)() for p, x in zip(pyus, xs)]
        else:
            objs = [p(lambda x=x: torch.from_numpy(x).cuda())() for p, x in zip(pyus, xs)]
        got = reveal(agg.sum(objs, axis=0))
        got = got.cpu().numpy() if isinstance(got, torch.Tensor) else got
        masked, ssum = ora.round(xs)
        assert np.array_equal(got, o.decode(ssum)), (mode, rnd)
        assert [int(v) for v in agg.last_digests[0].cpu().numpy().view(np.uint64)] == \
            [o.digest(m) for m in masked], (mode, rnd)
        if keep:
            for c in range(len(NAMES)):
                assert np.array_equal(agg.last_masked[0][c].cpu().numpy().view(np.uint64), masked[c]), (mode, rnd, c)
    # the pair stream consumed one raw draw more than the others
    assert agg._maskers["bob"].position("dave") == 2 * n + 1
    assert agg._maskers["dave"].position("bob") == 2 * n + 1
    assert agg._maskers["alice"].position("bob") == 2 * n


@pytest.mark.gpu
def test_layers_after_a_rejection_use_shifted_positions():
    """Two layers packed into one launch, the zero in the FIRST layer's
    range: the second layer's elements (later stream positions) follow the
    shifted stream too."""
    _gpu()
    from sfl_amd.device import PYU, reveal
    from sfl_amd.security.aggregation import SecureAggregator

    pair = _pair_states(("alice", "carol"), 7)
    pyus = [PYU(nm, 0) for nm in NAMES]
    agg = SecureAggregator(PYU("server", 0), pyus, seeds=pair, keep_masked=True)
    ora = o.OracleMaskers(NAMES, pair)
    rng = np.random.default_rng(3)
    layers = [[(rng.standard_normal(s) * 0.1).astype(np.float32) for s in (33, 17)] for _ in NAMES]
    got = reveal(agg.average([p(lambda d=d: d)() for p, d in zip(pyus, layers)], axis=0, weights=[1, 2, 3, 4]))
    flat = [np.concatenate(d) for d in layers]
    masked, ssum = ora.round(flat, weights=[1, 2, 3, 4])
    exp = o.decode(ssum, divisor=10)
    assert np.array_equal(np.concatenate(got), exp)
    for c in range(len(NAMES)):
        img = np.concatenate([agg.last_masked[li][c].cpu().numpy().view(np.uint64) for li in range(2)])
        assert np.array_equal(img, masked[c])


@pytest.mark.gpu
@pytest.mark.parametrize("host", [False, True])
def test_many_parties_rejection_replays_per_party(host):
    """10 co-located parties (the pair-shared many-client schedule): a raw 0
    on the (p03, p08) stream -- a pair drawn in a bipartite launch -- flags
    the round, which is replayed on the per-party path with numpy's
    rejection; this round and the next equal numpy's bit for bit, and the
    pair's position runs one raw draw ahead."""
    _gpu()
    from sfl_amd.device import PYU, reveal
    from sfl_amd.security.aggregation import SecureAggregator

    names = [f"p{c:02d}" for c in range(10)]
    seeds = o.seeds_for(names)
    pair = {(a, b): seeds[a][b] for a in names for b in names if a < b}
    pair[("p03", "p08")] = forced_zero_state(777)
    n = 2001
    pyus = [PYU(nm, 0) for nm in names]
    agg = SecureAggregator(PYU("server", 0), pyus, seeds=pair)
    ora = o.OracleMaskers(names, pair)
    rng = np.random.default_rng(12)
    for rnd in range(2):
        xs = [(rng.standard_normal(n) * 1e-2).astype(np.float32) for _ in names]
        objs = [p(lambda x=x: x if host else torch.from_numpy(x).cuda())() for p, x in zip(pyus, xs)]
        got = reveal(agg.sum(objs, axis=0))
        got = got.cpu().numpy() if isinstance(got, torch.Tensor) else got
        _, ssum = ora.round(xs)
        assert np.array_equal(got, o.decode(ssum)), (host, rnd)
    assert agg._maskers["p03"].position("p08") == 2 * n + 1
    assert agg._maskers["p00"].position("p01") == 2 * n
