"""Seeded random sweep of the SecureAggregator plugin against the oracle.

Each case draws a party count (2..10: the fused launch up to 8 co-located
parties, the per-party wire path beyond), a list of layers (possibly
zero-size, ragged shapes), a payload dtype per layer (float32 / float64 /
int64, numpy or torch), weights (none, python ints or floats, per-element
arrays), sum or average, and the plugin mode (fused / wire / keep_masked),
then runs three rounds and compares every decoded layer with the oracle's
float64 bit for bit, stream positions advancing layer by layer exactly as the
reference's per-layer ``rng.integers`` calls do.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import secagg as o  # noqa: E402

pytestmark = pytest.mark.gpu

N_CASES = 100


def _case(seed):
    rng = np.random.default_rng(1000 + seed)
    C = int(rng.integers(2, 11))
    nl = int(rng.integers(1, 5))
    shapes = []
    for _ in range(nl):
        r = rng.random()
        if r < 0.1:
            shapes.append((0,))
        elif r < 0.4:
            shapes.append((int(rng.integers(1, 2000)),))
        elif r < 0.8:
            shapes.append((int(rng.integers(1, 60)), int(rng.integers(1, 60))))
        else:
            shapes.append((int(rng.integers(1, 9)), int(rng.integers(1, 9)), int(rng.integers(1, 40))))
    # one dtype for every layer of this case when packed paths should be hit,
    # else a dtype per layer
    if rng.random() < 0.6:
        dts = [np.float32] * nl
    else:
        dts = [[np.float32, np.float64, np.int64][int(rng.integers(0, 3))] for _ in range(nl)]
    as_torch = bool(rng.random() < 0.35) and all(d == np.float32 for d in dts)
    wkind = ["none", "int", "float", "vec"][int(rng.integers(0, 4))]
    average = bool(rng.random() < 0.7)
    if not average:
        wkind = "none"
    if as_torch and wkind == "vec":
        wkind = "int"
    mode = ["fused", "wire", "keep"][int(rng.integers(0, 3))]
    return rng, C, shapes, dts, as_torch, wkind, average, mode


def _payload(rng, shape, dt, scale):
    if dt == np.int64:
        return rng.integers(-(1 << 16), 1 << 16, shape)
    return (rng.standard_normal(shape) * scale).astype(dt)


@pytest.mark.parametrize("seed", range(N_CASES))
def test_plugin_random_cases_match_oracle(seed):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.device import PYU, reveal as rv
    from sfl_amd.security.aggregation import SecureAggregator

    rng, C, shapes, dts, as_torch, wkind, average, mode = _case(seed)
    names = [f"p{int(v):03d}" for v in rng.permutation(C * 7)[:C]]
    seeds = o.seeds_for(names)
    pair = {(a, b): seeds[a][b] for a in names for b in names if a != b}
    pyus = [PYU(nm, 0) for nm in names]
    agg = SecureAggregator(PYU("server", 0), pyus, seeds=pair, fused=mode != "wire",
                           keep_masked=mode == "keep")
    offset = 0
    for rnd in range(3):
        data = [[_payload(rng, sh, dt, 10.0 ** rng.integers(-3, 2)) for sh, dt in zip(shapes, dts)]
                for _ in names]
        if wkind == "none":
            w = None
        elif wkind == "int":
            w = [int(v) for v in rng.integers(1, 100, C)]
        elif wkind == "float":
            w = [float(v) for v in rng.random(C) * 4 + 0.1]
        else:  # per-element weight arrays: drawn below, single-array payload
            w = None
        objs = []
        for p, d in zip(pyus, data):
            payload = [torch.from_numpy(a).to("cuda:0") for a in d] if as_torch else d
            objs.append(p(lambda x=payload: x)())
        if wkind == "vec":
            # per-element weights only for single-array payloads (np.average semantics)
            objs = [p(lambda x=d[0]: x)() for p, d in zip(pyus, data)]
            w = [rng.integers(1, 9, shapes[0]) for _ in names]
            got = rv(agg.average(objs, axis=0, weights=w))
            xs = [d[0] for d in data]
            exp, _, _ = o.secure_average(xs, names, weights=w, seeds=seeds, offset=offset)
            assert np.array_equal(got, exp.reshape(shapes[0])), (seed, rnd)
            offset += int(np.prod(shapes[0]))
            continue
        got = rv(agg.average(objs, axis=0, weights=w) if average else agg.sum(objs, axis=0))
        assert len(got) == len(shapes)
        for li, sh in enumerate(shapes):
            xs = [d[li] for d in data]
            if average:
                exp, s, masked = o.secure_average(xs, names, weights=w, seeds=seeds, offset=offset)
            else:
                exp, s, masked = o.secure_sum(xs, names, seeds=seeds, offset=offset)
            g = got[li].cpu().numpy() if as_torch else got[li]
            assert g.dtype == np.float64 and g.shape == sh, (seed, rnd, li)
            assert np.array_equal(g.reshape(-1), exp.reshape(-1)), (seed, rnd, li, mode, dts[li], wkind)
            if mode == "keep" and sh[0] != 0:
                for c in range(C):
                    mv = agg.last_masked[li][c].cpu().numpy().view(np.uint64)
                    assert np.array_equal(mv, masked[c].reshape(-1)), (seed, rnd, li, c)
            offset += int(np.prod(sh))


N_KERNEL_CASES = 60


@pytest.mark.parametrize("seed", range(N_KERNEL_CASES))
def test_fused_launch_random_shapes_match_oracle(seed):
    """``sa_fused_clients`` at random per-rank shapes: L local clients of T
    (L = 1..8, the other T - L as cross streams of every local client, fused
    or the per-client fallback), random n, stream offset up to 2^60, python
    float / int weights, gradients at random scales with a few values that
    force the exact int64 quantize path; digests, wire images and accumulate
    on or off.  The partial sum is the sum of the local clients' masked
    vectors of the oracle, bit for bit."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd import _lib as L
    from sfl_amd import kernels as K

    rng = np.random.default_rng(5000 + seed)
    T = int(rng.integers(2, 13))
    Lc = int(rng.integers(1, min(8, T) + 1))
    n = int(rng.choice([1, 2, 63, 64, 65, 1000, 4097, int(rng.integers(1, 200_000))]))
    offset = int(rng.integers(0, 1 << 60))
    names = [f"q{int(v):02d}" for v in rng.permutation(40)[:T]]
    seeds = o.seeds_for(names)
    scale = float(10.0 ** rng.integers(-4, 3))
    xs = [(rng.standard_normal(n) * scale).astype(np.float32) for _ in names]
    if n > 100 and rng.random() < 0.4:
        idx = rng.choice(n, 5, replace=False)
        xs[0][idx] = np.float32([3e9, -np.inf, np.nan, 1e30, -2.5e9])
    ws = ([float(v) for v in rng.random(T) * 3 + 0.05] if rng.random() < 0.5
          else [int(v) for v in rng.integers(1, 60, T)])
    masked = o.secure_masked(xs, names, weights=ws, seeds=seeds, offset=offset)
    local = list(range(Lc))
    remote = list(range(Lc, T))
    pg, ps = [], []
    for u in local:
        for v in local[u + 1:]:
            pg.append(L.pcg64_advance(L.pcg64_from_seed(seeds[names[u]][names[v]]), offset))
            ps.append(1 if names[v] > names[u] else -1)
    cross = []
    for u in local:
        for v in remote:
            cross.append((L.pcg64_advance(L.pcg64_from_seed(seeds[names[u]][names[v]]), offset),
                          1 if names[v] > names[u] else -1, v))
    want_dig, want_mo, acc = (bool(rng.random() < 0.5) for _ in range(3))
    base = rng.integers(0, 2**63, n).astype(np.uint64) if acc else np.zeros(n, np.uint64)
    s = torch.from_numpy(base.view(np.int64).copy()).to("cuda:0")
    dig = torch.zeros(Lc, dtype=torch.int64, device="cuda:0") if want_dig else None
    mo = [torch.empty(n, dtype=torch.int64, device="cuda:0") for _ in local] if want_mo else None
    flags = torch.zeros(1, dtype=torch.int32, device="cuda:0")
    K.fused_clients([torch.from_numpy(xs[u]).to("cuda:0") for u in local], [ws[u] for u in local], pg, ps,
                    cross, len(remote), s, accumulate=acc, digests=dig, flags=flags, masked_outs=mo)
    torch.cuda.synchronize()
    exp = base.copy()
    for u in local:
        exp = exp + masked[u]
    ctx = (seed, T, Lc, n, want_dig, want_mo, acc)
    assert np.array_equal(K.as_u64(s), exp), ctx
    if want_mo:
        for u in local:
            assert np.array_equal(K.as_u64(mo[u]), masked[u]), ctx + (u,)
    if want_dig:
        assert [int(v) for v in K.as_u64(dig)] == [o.digest(masked[u]) for u in local], ctx
    assert int(flags.item()) == 0


N_MANY_CASES = 24


@pytest.mark.parametrize("seed", range(N_MANY_CASES))
def test_many_clients_random_cases_match_oracle(seed):
    """The pair-shared many-client schedule (kernels.fused_many) on random
    shapes: 9..40 co-located clients (short last quads and groups included),
    random n, stream offsets up to 2^50, python-int weights, random names
    (mixed pair signs), sum written or accumulated: equal to the oracle's
    server sum bit for bit, and to the per-client path."""
    from sfl_amd import _lib as L
    from sfl_amd import kernels as K

    rng = np.random.default_rng(5000 + seed)
    C = int(rng.integers(9, 41))
    n = int(rng.integers(1, 50_000))
    offset = int(rng.integers(0, 1 << 50))
    names = [f"n{int(v):05d}" for v in rng.permutation(100_000)[:C]]
    seeds = o.seeds_for(names)
    w = [int(v) for v in rng.integers(1, 50, C)]
    xs = [(rng.standard_normal(n) * 0.05).astype(np.float32) for _ in range(C)]
    pg, ps = [], []
    for u in range(C):
        for v in range(u + 1, C):
            pg.append(L.pcg64_advance(L.pcg64_from_seed(seeds[names[u]][names[v]]), offset))
            ps.append(1 if names[v] > names[u] else -1)
    exp = o.server_sum(o.secure_masked(xs, names, weights=w, seeds=seeds, offset=offset))
    dev = torch.device("cuda", 0)
    xt = [torch.from_numpy(x).to(dev) for x in xs]
    accumulate = bool(rng.integers(0, 2))
    base = rng.integers(0, 2**64 - 1, n, dtype=np.uint64) if accumulate else np.zeros(n, dtype=np.uint64)
    s = torch.from_numpy(base.view(np.int64).copy()).to(dev)
    K.fused_many(xt, [float(v) for v in w], pg, ps, s, accumulate=accumulate)
    s2 = torch.empty(n, dtype=torch.int64, device=dev)
    K.fused_clients(xt, [float(v) for v in w], pg, ps, [], 0, s2, digests=torch.zeros(C, dtype=torch.int64, device=dev))
    torch.cuda.synchronize()
    assert np.array_equal(K.as_u64(s), base + exp), (C, n)
    assert np.array_equal(K.as_u64(s2), exp), (C, n)
