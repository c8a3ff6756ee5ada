"""DP pre-step on the GPU vs the oracle (oracle/dp.py):
norm reduction, clip (exact), Philox noise (within float tolerance of the
numpy restatement), and the fused sa_mask_dp == perturb-then-mask bit for bit."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
from oracle import dp as D  # noqa: E402
from oracle import secagg as o  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _K():
    from sfl_amd import kernels as K

    return K


def _sumsq(x):
    from sfl_amd import _lib as L

    out = torch.zeros(1, dtype=torch.float64, device=DEV)
    part = torch.empty(L.SA_DP_PARTIALS, dtype=torch.float64, device=DEV)
    return _K().sumsq_f32(x, out, part)


@pytest.mark.parametrize("n", [1, 3, 4, 1027, 1_000_003])
def test_sumsq_deterministic_and_accurate(n):
    """sa_sumsq_f32 = the layer's np.linalg.norm(x) ** 2 as the reference
    forms it under numpy 1.23.5 (oracle layer_sq_norm: the float32 norm
    squared in float64), deterministic; accumulating two layers adds in
    float64 (the reference's python sum)."""
    x = torch.randn(n, device=DEV)
    a, b = _sumsq(x), _sumsq(x)
    torch.cuda.synchronize()
    assert torch.equal(a, b)
    xh = x.cpu().numpy()
    assert a.item() == float(D.layer_sq_norm(xh))
    nrm = np.sqrt(a.item())
    assert np.float32(nrm) == nrm and nrm * nrm == a.item()  # the exact square of a float32 norm
    from sfl_amd import _lib as L

    part = torch.empty(L.SA_DP_PARTIALS, dtype=torch.float64, device=DEV)
    y = torch.randn(n + 5, device=DEV)
    _K().sumsq_f32(y, a, part, accumulate=True)
    assert a.item() == float(D.global_sq([xh, y.cpu().numpy()]))


@pytest.mark.parametrize("clip", [0.5, 1e6])
def test_perturb_clip_exact_without_noise(clip):
    K = _K()
    n = 70_001
    x = torch.randn(n, device=DEV) * 3
    s = _sumsq(x)
    dp = K.make_dp(s, l2_norm_clip=clip, noise_std=0.0, num_updates=4, key=1)
    y = K.dp_perturb(x, torch.empty_like(x), dp)
    torch.cuda.synchronize()
    scale = D.clip_scale(s.item(), clip)
    assert np.array_equal(y.cpu().numpy(), x.cpu().numpy() * scale)


@pytest.mark.parametrize("n", [1, 3, 4, 5, 1023, 1024, 1025, 4095, 4096, 4097, 262_147])
def test_perturb_tile_edges_and_no_write_past_n(n):
    """The tile form's whole-tile and partial-tile paths (1,024 elements per
    workgroup) against the oracle's noise stream; the 16 floats after n keep
    their sentinel."""
    K = _K()
    key, ctr = 0x0123456789ABCDEF, 4 * 7
    x = torch.randn(n, device=DEV) * 0.2
    s = _sumsq(x)
    buf = torch.full((n + 16,), 12345.0, device=DEV)
    dp = K.make_dp(s, l2_norm_clip=0.5, noise_std=0.3, num_updates=4, key=key, counter0=ctr)
    K.dp_perturb(x, buf[:n], dp)
    torch.cuda.synchronize()
    assert torch.all(buf[n:] == 12345.0)
    xh = x.cpu().numpy()
    exp = D.perturb(xh, D.clip_scale(s.item(), 0.5), D.gauss(key, ctr, n), 0.3, 4)
    assert np.allclose(buf[:n].cpu().numpy(), exp, rtol=2e-5, atol=2e-6)


@pytest.mark.parametrize("updates", [4, 3])
def test_perturb_noise_matches_oracle_stream(updates):
    K = _K()
    n, key, ctr = 100_003, 0xDEADBEEF12345678, 4 * 1000
    x = torch.zeros(n, device=DEV)
    s = _sumsq(torch.ones(4, device=DEV))
    dp = K.make_dp(s, l2_norm_clip=1.0, noise_std=1.5, num_updates=updates, key=key, counter0=ctr)
    y = K.dp_perturb(x, torch.empty_like(x), dp).cpu().numpy()
    z = D.gauss(key, ctr, n)
    exp = D.perturb(np.zeros(n, np.float32), 1.0, z, 1.5, updates)
    assert np.allclose(y, exp, rtol=2e-5, atol=2e-6)
    assert abs(y.mean()) < 0.01 and abs(y.std() - 1.5 / updates) < 0.01


@pytest.mark.parametrize("nstreams,updates", [(0, 8), (3, 8), (17, 8), (3, 3), (7, 6)])
def test_fused_mask_dp_equals_perturb_then_mask(nstreams, updates):
    K, L = _K(), None
    from sfl_amd import _lib as L

    n = 50_003
    x = torch.randn(n, device=DEV) * 0.05
    s = _sumsq(x)
    seeds = [o.pair_seed(0, j + 1) for j in range(nstreams)]
    streams = [(L.pcg64_from_seed(sd), 1 if j % 2 else -1, j) for j, sd in enumerate(seeds)]
    # num_updates a power of two: the kernels multiply by the exact reciprocal; else IEEE division
    mk = lambda: K.make_dp(s, l2_norm_clip=0.3, noise_std=0.01, num_updates=updates, key=77, counter0=40)  # noqa: E731
    xp = K.dp_perturb(x, torch.empty_like(x), mk())
    m1 = torch.empty(n, dtype=torch.int64, device=DEV)
    d1 = torch.zeros(1, dtype=torch.int64, device=DEV)
    K.mask(xp, m1, streams, weight=3.0, digest=d1)
    m2 = torch.empty(n, dtype=torch.int64, device=DEV)
    d2 = torch.zeros(1, dtype=torch.int64, device=DEV)
    K.mask_dp(x, m2, streams, mk(), weight=3.0, digest=d2)
    torch.cuda.synchronize()
    bad = (m1 != m2).nonzero().flatten()
    assert bad.numel() == 0, f"{bad.numel()} masked elements differ, first {bad[:8].tolist()}"
    assert torch.equal(d1, d2)
    # and the masked vector is the oracle's for the perturbed input
    exp = o.quantize(xp.cpu().numpy(), 3)
    for sd, (_, sg, _) in zip(seeds, streams):
        mm = o.mask_stream(sd, n)
        exp = exp + mm if sg > 0 else exp - mm
    assert np.array_equal(m2.cpu().numpy().view(np.uint64), exp)


@pytest.mark.parametrize("each_layer", [False, True])
def test_gaussian_model_dp_class_vs_oracle(each_layer):
    from sfl_amd.security.privacy import GaussianModelDP

    rng = np.random.default_rng(5)
    layers = [rng.standard_normal((50, 4)).astype(np.float32), rng.standard_normal(50).astype(np.float32),
              rng.standard_normal((3, 50)).astype(np.float32)]
    dp = GaussianModelDP(noise_multiplier=0.7, num_clients=8, l2_norm_clip=2.0, is_clip_each_layer=each_layer,
                         seed=99)
    got = dp(layers)
    exp = D.gaussian_model_dp(layers, 0.7, 8, 2.0, key=99, is_clip_each_layer=each_layer)
    for g, e, a in zip(got, exp, layers):
        assert isinstance(g, np.ndarray) and g.dtype == np.float32 and g.shape == a.shape
        assert np.allclose(g, e, rtol=1e-5, atol=1e-6)
    # noise-free: exact clip
    dp0 = GaussianModelDP(noise_multiplier=0.0, num_clients=8, l2_norm_clip=2.0, seed=1)
    got0 = dp0(layers)
    exp0 = D.gaussian_model_dp(layers, 0.0, 8, 2.0)
    for g, e in zip(got0, exp0):
        assert np.array_equal(g, e)


def _reference_clip_numpy(inputs, clip, each_layer):
    """mechanism_fl.py:71-108 with noise_multiplier = 0, restated on numpy's
    own float32 arithmetic (np.linalg.norm per layer, ** 2, python sum,
    np.sqrt, min(1, clip / norm), the float32 array times the scale).  Runs
    under this image's numpy 2 (NEP 50: clip / float32 divides in float32,
    where the reference's numpy 1.23.5 divides in float64 -- within one ulp
    of the scale)."""
    def gnorm(arrs):
        return np.sqrt(sum([np.linalg.norm(a) ** 2 for a in arrs]))

    norm_all = gnorm(inputs)
    if each_layer:
        return [a * min(1, clip / np.sqrt(gnorm([a]) * norm_all)) for a in inputs]
    scale = min(1, clip / norm_all)
    return [a * scale for a in inputs]


@pytest.mark.parametrize("each_layer", [False, True])
@pytest.mark.parametrize("clip", [0.5, 1e6])
def test_gaussian_model_dp_vs_reference_numpy_clip(each_layer, clip):
    """GaussianModelDP with noise_multiplier = 0 against
    the reference's clip evaluated by numpy itself.  The device forms the
    norm with the reference's float32 structure (sa_sumsq_f32); what is left
    is the reference's BLAS float32 dot, whose accumulation error the test
    measures (|np.linalg.norm - exact| / exact) and allows, plus 4 ulps of
    float32 for the scale's division and the product.  With no clipping
    (clip 1e6: scale 1) the output is the input bit for bit."""
    from sfl_amd.security.privacy import GaussianModelDP

    rng = np.random.default_rng(17)
    layers = [(rng.standard_normal(s) * 0.05).astype(np.float32) for s in ((300, 200), (200,), (200, 10), (10,))]
    layers.append((rng.standard_normal(1_000_003) * 0.01).astype(np.float32))
    dp = GaussianModelDP(noise_multiplier=0.0, num_clients=8, l2_norm_clip=clip, is_clip_each_layer=each_layer,
                         seed=3)
    got = dp(layers)
    ref = _reference_clip_numpy(layers, clip, each_layer)
    exact = [np.sqrt(np.sum(a.astype(np.float64) ** 2)) for a in layers]
    blas_rel = max(abs(float(np.linalg.norm(a)) - e) / e for a, e in zip(layers, exact))
    tot_exact = np.sqrt(sum(e * e for e in exact))
    blas_rel = max(blas_rel, abs(float(np.sqrt(sum([np.linalg.norm(a) ** 2 for a in layers]))) - tot_exact) / tot_exact)
    tol = 2 * blas_rel + 4 * 2.0**-24
    for g, r, a in zip(got, ref, layers):
        assert g.dtype == np.float32 and r.dtype == np.float32
        if clip == 1e6:
            assert np.array_equal(g, a) and np.array_equal(r, a)
        else:
            np.testing.assert_allclose(g, r, rtol=tol, atol=0)


def test_loopback_client_dp_round_vs_oracle():
    """LoopbackClient.submit(dp=...) with in-process parties over 127.0.0.1:
    every client perturbs its device copy (GaussianModelDP: clip to the
    global norm + Philox noise) and masks it; the server's decoded sum equals
    the oracle's sum of the perturbed vectors bit for bit (the noise taken
    from the standalone perturb kernel, which test_fused_mask_dp_equals_
    perturb_then_mask pins to the fused kernel)."""
    import threading

    from sfl_amd.loopback import LoopbackClient, LoopbackServer
    from sfl_amd.security.privacy import GaussianModelDP

    K = _K()
    names, n = ["p0", "p1", "p2"], 30_011
    seeds = o.seeds_for(names)
    rng = np.random.default_rng(9)
    xs = [(rng.standard_normal(n) * 0.05).astype(np.float32) for _ in names]
    srv = LoopbackServer(len(names))
    res = {}

    def client(i):
        cl = LoopbackClient(names[i], i, srv.port, seeds={v: seeds[names[i]][v] for v in names if v != names[i]})
        cl.handshake()
        dp = GaussianModelDP(noise_multiplier=0.5, num_clients=3, l2_norm_clip=0.8, seed=100 + i)
        out = np.empty(n, dtype=np.float64)
        cl.submit(xs[i], 0, dp=dp, result_into=out)
        res[i] = (cl.result(n), cl.last_result_xor)
        cl.close()

    ts = [threading.Thread(target=client, args=(i,)) for i in range(len(names))]
    for t in ts:
        t.start()
    srv.accept(timeout=60)
    got, _ = srv.round(n, 0)
    for t in ts:
        t.join(60)
    srv.close()
    # the expected perturbed inputs, from the same DP parameters
    xp = []
    for i, x in enumerate(xs):
        dp = GaussianModelDP(noise_multiplier=0.5, num_clients=3, l2_norm_clip=0.8, seed=100 + i)
        d = torch.from_numpy(x).to(DEV)
        xp.append(K.dp_perturb(d, torch.empty_like(d), dp.params(dp.sumsq([d]), n)).cpu().numpy())
    exp = o.secure_sum(xp, names, seeds=seeds)[0]
    assert np.array_equal(got, exp)
    for i in range(len(names)):
        assert np.array_equal(res[i][0], exp)
        assert res[i][1] == int(np.bitwise_xor.reduce(exp.view(np.uint64)))
    assert float(np.abs(exp - np.sum(xs, axis=0)).max()) > 1e-4  # the noise is there
