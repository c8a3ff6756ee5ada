"""The SecureAggregator plugin surface on the HIP path.

Mirrors the reference's AggregatorBase contract
(tests/security/aggregation/test_aggregator_base.py:20-160: alice and bob
hold data, carol aggregates) and checks the notebook KAT
(docs/developer/algorithm/secure_aggregation.ipynb cells 17-18) through the
full plugin: quantize + mask on the parties, sum + decode on the server.
"""
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import secagg as o  # noqa: E402

pytestmark = pytest.mark.gpu


class _Env:
    def __init__(self):
        from sfl_amd.device import PYU

        self.alice, self.bob, self.carol = PYU("alice", 0), PYU("bob", 0), PYU("carol", 0)


@pytest.fixture(params=["fused", "wire"])
def env_and_aggregator(request):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.security.aggregation import SecureAggregator

    env = _Env()
    agg = SecureAggregator(env.carol, [env.alice, env.bob], fused=request.param == "fused")
    return env, agg


def reveal(x):
    from sfl_amd.device import reveal as r

    return r(x)


class TestAggregatorContract:
    def test_sum_on_single_should_ok(self, env_and_aggregator):
        env, aggregator = env_and_aggregator
        a = env.alice(lambda: np.array([[1.0, 2.0, 3], [4.0, 5.0, 6.0]]))()
        b = env.bob(lambda: np.array([[11.0, 12.0, 13.0], [14, 15.0, 16.0]]))()
        sum_val = reveal(aggregator.sum([a, b], axis=0))
        np.testing.assert_almost_equal(sum_val, np.array([[12.0, 14.0, 16.0], [18.0, 20.0, 22.0]]), decimal=5)

    def test_sum_on_list_should_ok(self, env_and_aggregator):
        env, aggregator = env_and_aggregator
        a = env.alice(lambda: [np.array([[1, 2, 3], [4, 5, 6]]), np.array([[21, 22, 23], [24, 25, 26]])])()
        b = env.bob(lambda: [np.array([[11, 12, 13], [14, 15, 16]]), np.array([[31, 32, 33], [34, 35, 36]])])()
        sum_val = reveal(aggregator.sum([a, b], axis=0))
        np.testing.assert_almost_equal(sum_val[0], np.array([[12, 14, 16], [18, 20, 22]]), decimal=5)
        np.testing.assert_almost_equal(sum_val[1], np.array([[52, 54, 56], [58, 60, 62]]), decimal=5)

    def test_average_on_single_without_weights_should_ok(self, env_and_aggregator):
        env, aggregator = env_and_aggregator
        a = env.alice(lambda: np.array([[1.0, 2.0, 3.0], [4.0, 5.0, 6.0]]))()
        b = env.bob(lambda: np.array([[11.0, 12.0, 13.0], [14.0, 15.0, 16.0]]))()
        avg = reveal(aggregator.average([a, b], axis=0))
        np.testing.assert_almost_equal(avg, np.array([[6.0, 7.0, 8.0], [9.0, 10.0, 11.0]]), decimal=5)

    def test_average_on_list_without_weights_should_ok(self, env_and_aggregator):
        env, aggregator = env_and_aggregator
        a = env.alice(lambda: [np.array([[1, 2, 3], [4, 5, 6]]), np.array([[21, 22, 23], [24, 25, 26]])])()
        b = env.bob(lambda: [np.array([[11, 12, 13], [14, 15, 16]]), np.array([[31, 32, 33], [34, 35, 36]])])()
        avg = reveal(aggregator.average([a, b], axis=0))
        np.testing.assert_almost_equal(avg[0], np.array([[6, 7, 8], [9, 10, 11]]), decimal=5)
        np.testing.assert_almost_equal(avg[1], np.array([[26, 27, 28], [29, 30, 31]]), decimal=5)

    def test_average_with_weights_should_ok(self, env_and_aggregator):
        env, aggregator = env_and_aggregator
        a = env.alice(lambda: np.array([[1, 2, 3], [4, 5, 6]]))()
        b = env.bob(lambda: np.array([[11, 12, 13], [14, 15, 16]]))()
        avg_val = reveal(aggregator.average([a, b], axis=0, weights=[2, 3]))
        np.testing.assert_almost_equal(avg_val, np.array([[7, 8, 9], [10, 11, 12]]), decimal=4)

    def test_average_on_list_with_weights_should_ok(self, env_and_aggregator):
        env, aggregator = env_and_aggregator
        a = env.alice(lambda: [np.array([[1, 2, 3], [4, 5, 6]]), np.array([[21, 22, 23], [24, 25, 26]])])()
        b = env.bob(lambda: [np.array([[11, 12, 13], [14, 15, 16]]), np.array([[31, 32, 33], [34, 35, 36]])])()
        avg = reveal(aggregator.average([a, b], axis=0, weights=[2, 3]))
        np.testing.assert_almost_equal(avg[0], np.array([[7, 8, 9], [10, 11, 12]]), decimal=4)
        np.testing.assert_almost_equal(avg[1], np.array([[27, 28, 29], [30, 31, 32]]), decimal=4)

    def test_average_with_same_shape_weights_should_ok(self, env_and_aggregator):
        env, aggregator = env_and_aggregator
        arr0 = np.array([[1, 2, 3]])
        arr1 = np.array([[11, 12, 13]])
        a = env.alice(lambda: arr0)()
        b = env.bob(lambda: arr1)()
        weights = np.array([[[5, 7, 2]], [[5, 3, 8]]])
        avg_val = reveal(aggregator.average([a, b], axis=0, weights=weights))
        np.testing.assert_almost_equal(avg_val, np.average([arr0, arr1], axis=0, weights=weights), decimal=4)


def test_notebook_kat_through_the_plugin():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.device import PYU, reveal as rv
    from sfl_amd.security.aggregation import SecureAggregator

    here = os.path.join(os.path.dirname(__file__), "golden", "notebook_kat.json")
    k = json.load(open(here))
    alice, bob = PYU("alice", 0), PYU("bob", 0)
    agg = SecureAggregator(device=alice, participants=[alice, bob])
    a = alice(lambda: np.array(k["arr0"]))()
    b = bob(lambda: np.array(k["arr1"]))()
    s = rv(agg.sum([a, b], axis=0))
    avg = rv(agg.average([a, b], axis=0))
    assert s.dtype == np.float64
    assert np.abs(s - np.array(k["secure_sum"])).max() < 1e-8
    assert np.abs(avg - np.array(k["secure_average"])).max() < 1e-8


@pytest.mark.parametrize("dtype", [np.float64, np.float32])
def test_config1_two_parties_1m_bit_exact(dtype):
    """BASELINE config 1's shape through the plugin: 2 parties, a 1M-element
    numpy vector each (np.random.rand-style like the KAT), sum then average
    (consecutive stream positions): decoded float64 equal to the oracle bit
    for bit, and within the stated tolerance of the float sum (|err| <
    C * 2^-fxp for the sum, / C for the average)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.device import PYU, reveal as rv
    from sfl_amd.security.aggregation import SecureAggregator

    names, n = ["alice", "bob"], 1_000_000
    seeds = o.seeds_for(names)
    pyus = [PYU(nm, 0) for nm in names]
    agg = SecureAggregator(pyus[0], pyus, seeds={("alice", "bob"): seeds["alice"]["bob"]})
    rng = np.random.default_rng(11)
    xs = [rng.random(n).astype(dtype) for _ in names]
    objs = [p(lambda x=x: x)() for p, x in zip(pyus, xs)]
    s = rv(agg.sum(objs, axis=0))
    avg = rv(agg.average(objs, axis=0))
    assert s.dtype == np.float64 and avg.dtype == np.float64
    assert np.array_equal(s, o.secure_sum(xs, names, seeds=seeds)[0])
    assert np.array_equal(avg, o.secure_average(xs, names, seeds=seeds, offset=n)[0])
    fsum = xs[0].astype(np.float64) + xs[1]
    assert np.abs(s - fsum).max() < 2 * 2.0**-18
    assert np.abs(avg - fsum / 2).max() < 2.0**-18


@pytest.mark.parametrize("fused,keep", [(True, False), (False, True), (True, True)])
def test_rounds_match_oracle_bit_exact(fused, keep):
    """Several FL-style rounds with explicit seeds: decoded results equal the
    oracle's float64 bit for bit, and the per-party masked vectors (wire
    images) equal the oracle's, round after round (stream positions advance).
    fused + keep: the fused launch (pair streams expanded once) stores the
    wire images; not fused: one sa_mask launch per party."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.device import PYU, reveal as rv
    from sfl_amd.security.aggregation import SecureAggregator

    names = ["alice", "bob", "carol", "dave"]
    seeds = o.seeds_for(names)
    pair = {(a, b): seeds[a][b] for a in names for b in names if a != b}
    pyus = [PYU(nm, 0) for nm in names]
    server = PYU("server", 0)
    agg = SecureAggregator(server, pyus, seeds=pair, fused=fused, keep_masked=keep)
    rng = np.random.default_rng(4)
    offset = 0
    for rnd in range(3):
        layers = [(rng.standard_normal((3, 5)) * 0.1).astype(np.float32), rng.standard_normal(7).astype(np.float32)]
        data = [[(l_ + 0.01 * i).astype(np.float32) for l_ in layers] for i in range(len(names))]
        objs = [p(lambda d=d: d)() for p, d in zip(pyus, data)]
        w = [10 * (i + 1) for i in range(len(names))]
        got = rv(agg.average(objs, axis=0, weights=w))
        for li in range(2):
            xs = [d[li] for d in data]
            exp, s, masked = o.secure_average(xs, names, weights=w, seeds=seeds, offset=offset)
            assert np.array_equal(got[li], exp.reshape(xs[0].shape)), (rnd, li)
            if keep:
                for c in range(len(names)):
                    assert np.array_equal(agg.last_masked[li][c].cpu().numpy().view(np.uint64), masked[c].reshape(-1))
            offset += xs[0].size
        if keep:
            assert len(agg.last_masked) == 2


def test_torch_payload_stays_on_device():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.device import PYU, reveal as rv
    from sfl_amd.security.aggregation import SecureAggregator

    ps = [PYU(f"c{i}", 0) for i in range(3)]
    agg = SecureAggregator(PYU("srv", 0), ps)
    ts = [torch.randn(1000, device="cuda:0") for _ in ps]
    out = rv(agg.sum([p(lambda t=t: t)() for p, t in zip(ps, ts)], axis=0))
    assert isinstance(out, torch.Tensor) and out.is_cuda and out.dtype == torch.float64
    assert float((out - torch.stack(ts).double().sum(0)).abs().max()) < 3 * 2.0**-18


def test_single_participant_and_errors():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.device import PYU, reveal as rv
    from sfl_amd.security.aggregation import SecureAggregator

    a = PYU("alice", 0)
    agg = SecureAggregator(a, [a])
    x = np.float32([1.5, -2.25, 3e-6])
    got = rv(agg.sum([a(lambda: x)()], axis=0))
    assert np.array_equal(got, o.decode(o.quantize(x)))
    with pytest.raises(AssertionError, match="should not be None or empty"):
        agg.sum([], axis=0)
    b = PYU("bob", 0)
    agg2 = SecureAggregator(a, [a, b])
    with pytest.raises(AssertionError):
        agg2.sum([a(lambda: x)()], axis=0)  # dropout is not supported


def test_homo_binning_style_integer_sums():
    """Secondary caller: HomoBinning sums per-party
    int64 missing counts and [cols x split-points] rank tables with
    aggregator.sum (sfl/preprocessing/binning/homo_binning.py:143-167,
    homo_binning_base.py:133-144, 208-224).  Integer data stays int64 through
    quantization, so the decoded sums are exact."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.device import PYU, reveal as rv
    from sfl_amd.security.aggregation import SecureAggregator

    parties = [PYU(n, 0) for n in ("alice", "bob", "carol")]
    agg = SecureAggregator(PYU("server", 0), parties)
    rng = np.random.default_rng(11)
    for it in range(5):
        missing = [rng.integers(0, 1000, 9) for _ in parties]
        ranks = [rng.integers(0, 10**6, (9, 11)) for _ in parties]
        got_m = rv(agg.sum([p(lambda a=a: a)() for p, a in zip(parties, missing)], axis=0))
        got_r = rv(agg.sum([p(lambda a=a: a)() for p, a in zip(parties, ranks)], axis=0))
        assert np.array_equal(got_m, np.sum(missing, axis=0).astype(np.float64))
        assert np.array_equal(got_r, np.sum(ranks, axis=0).astype(np.float64))


def test_subclass_with_reference_constructor_contract():
    """StatefulFedGenAggregator subclasses SecureAggregator as
    (device, participants, fxp_bits) and calls super().average(data, axis,
    None) (sfl/security/aggregation/stateful_fedgen_aggregator.py:23-60)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.device import PYU, reveal as rv
    from sfl_amd.security.aggregation import SecureAggregator

    class StatefulFedGenLike(SecureAggregator):
        def __init__(self, device, participants, server_actor, fxp_bits: int = 18):
            super().__init__(device, participants, fxp_bits)
            self.server_actor = server_actor

        def average(self, data, axis=None, weights=None):
            avg = super().average(data, axis, None)
            if weights is not None:
                return self._device(lambda x: x)({"generator_params": self.server_actor, "model_params": avg})
            return avg

    parties = [PYU("a", 0), PYU("b", 0)]
    agg = StatefulFedGenLike(PYU("s", 0), parties, "gen-weights", 18)
    xs = [np.arange(6, dtype=np.float32) * (i + 1) for i in range(2)]
    out = rv(agg.average([p(lambda x=x: x)() for p, x in zip(parties, xs)], axis=0, weights=[1, 1]))
    assert out["generator_params"] == "gen-weights"
    # the subclass averages with weights=None (stateful_fedgen_aggregator.py:59):
    # bit-exact vs the oracle's unweighted secure average (PRG-independent)
    exp = o.secure_average(xs, ["a", "b"])[0]
    assert np.array_equal(rv(out["model_params"]), exp)
    assert np.allclose(exp, (xs[0] + xs[1]) / 2, atol=2 * 2.0**-18)


@pytest.mark.parametrize("as_list", [False, True])
def test_numpy_scalar_weights_numpy_1_23_semantics(as_list):
    """numpy-scalar weights on float32 payloads: float32 arithmetic with the
    weight rounded to float32, as numpy 1.23.5 (the reference's pinned
    version, uv.lock:1189-1190) computes x * w; bit-exact vs the oracle."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.device import PYU, reveal as rv
    from sfl_amd.security.aggregation import SecureAggregator

    names = ["alice", "bob", "carol"]
    seeds = o.seeds_for(names)
    pair = {(a, b): seeds[a][b] for a in names for b in names if a != b}
    pyus = [PYU(nm, 0) for nm in names]
    agg = SecureAggregator(PYU("server", 0), pyus, seeds=pair)
    rng = np.random.default_rng(8)
    xs = [(rng.standard_normal(1001) * 0.1).astype(np.float32) for _ in names]
    w = [np.float64(1.3), np.int64(3), np.float32(0.7)]
    objs = [p(lambda x=x: [x] if as_list else x)() for p, x in zip(pyus, xs)]
    got = rv(agg.average(objs, axis=0, weights=w))
    got = got[0] if as_list else got
    exp, _, _ = o.secure_average(xs, names, weights=w, seeds=seeds)
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("fused", [True, False])
def test_zero_size_and_ragged_layers(fused):
    """Empty arrays (alone and as one layer of a list) aggregate to empty
    float64 arrays of the same shape; the other layers and the stream
    positions are unaffected (the next round still matches the oracle)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.device import PYU, reveal as rv
    from sfl_amd.security.aggregation import SecureAggregator

    names = ["alice", "bob", "carol"]
    seeds = o.seeds_for(names)
    pair = {(a, b): seeds[a][b] for a in names for b in names if a != b}
    pyus = [PYU(nm, 0) for nm in names]
    agg = SecureAggregator(PYU("server", 0), pyus, seeds=pair, fused=fused)
    e = rv(agg.sum([p(lambda: np.zeros((0, 3), np.float32))() for p in pyus], axis=0))
    assert e.shape == (0, 3) and e.dtype == np.float64
    rng = np.random.default_rng(2)
    data = [[np.zeros(0, np.float32), (rng.standard_normal(5) * 0.1).astype(np.float32)] for _ in names]
    got = rv(agg.sum([p(lambda d=d: d)() for p, d in zip(pyus, data)], axis=0))
    assert got[0].shape == (0,)
    exp, _, _ = o.secure_sum([d[1] for d in data], names, seeds=seeds)
    assert np.array_equal(got[1], exp)
    xs = [(rng.standard_normal(9) * 0.1).astype(np.float32) for _ in names]
    got = rv(agg.sum([p(lambda x=x: x)() for p, x in zip(pyus, xs)], axis=0))
    exp, _, _ = o.secure_sum(xs, names, seeds=seeds, offset=5)
    assert np.array_equal(got, exp)


@pytest.mark.parametrize("as_torch", [False, True])
def test_many_colocated_parties_pair_shared(as_torch):
    """12 / 13 parties on one GPU (more than one fused launch holds): the
    plugin takes the pair-shared schedule (every pair stream expanded once);
    three weighted rounds, numpy (host latency path) or torch payloads, equal
    the oracle's decoded averages bit for bit at the advancing stream
    positions."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.device import PYU, reveal as rv
    from sfl_amd.security.aggregation import SecureAggregator

    C = 13 if as_torch else 12
    names = [f"p{c:02d}" for c in range(C)][::-1]
    seeds = o.seeds_for(names)
    pyus = [PYU(nm, 0) for nm in names]
    agg = SecureAggregator(PYU("server", 0), pyus,
                           seeds={(a, b): seeds[a][b] for a in names for b in names if a < b})
    rng = np.random.default_rng(C)
    offset = 0
    for rnd in range(3):
        xs = [(rng.standard_normal(1001) * 0.1).astype(np.float32) for _ in names]
        w = [3 * c + rnd + 1 for c in range(C)]
        objs = [p(lambda x=x: torch.from_numpy(x).cuda() if as_torch else x)() for p, x in zip(pyus, xs)]
        got = rv(agg.average(objs, axis=0, weights=w))
        got = got.cpu().numpy() if as_torch else got
        exp = o.secure_average(xs, names, weights=w, seeds=seeds, offset=offset)[0]
        assert np.array_equal(got, exp), rnd
        offset += xs[0].size


@pytest.mark.parametrize("dtype,n", [(np.float32, 262_144), (np.float32, 262_148), (np.float64, 131_072),
                                     (np.float64, 131_073), (np.int64, 131_072), (np.int64, 131_073)])
def test_small_call_boundary_bit_exact(dtype, n):
    """Both sides of SMALL_CALL_BYTES (1 MiB a party): the pinned one-copy
    path and the direct-copy path, 3 parties, sum then weighted average
    (consecutive stream positions), then a small call again on the same
    aggregator (staging reused across sizes) -- bit-exact vs the oracle."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.device import PYU, reveal as rv
    from sfl_amd.security.aggregation import SecureAggregator

    names = ["alice", "bob", "carol"]
    seeds = o.seeds_for(names)
    pyus = [PYU(nm, 0) for nm in names]
    agg = SecureAggregator(PYU("server", 0), pyus,
                           seeds={(a, b): seeds[a][b] for a in names for b in names if a < b})
    rng = np.random.default_rng(n)
    mk = (lambda m: (rng.standard_normal(m) * 3).astype(dtype)) if dtype != np.int64 else \
        (lambda m: rng.integers(-10**6, 10**6, m))
    xs = [mk(n) for _ in names]
    ws = [2, 3, 5]
    objs = [p(lambda x=x: x)() for p, x in zip(pyus, xs)]
    s = rv(agg.sum(objs, axis=0))
    assert np.array_equal(s, o.secure_sum(xs, names, seeds=seeds)[0])
    avg = rv(agg.average(objs, axis=0, weights=ws))
    assert np.array_equal(avg, o.secure_average(xs, names, weights=ws, seeds=seeds, offset=n)[0])
    ys = [mk(99) for _ in names]
    s2 = rv(agg.sum([p(lambda y=y: y)() for p, y in zip(pyus, ys)], axis=0))
    assert np.array_equal(s2, o.secure_sum(ys, names, seeds=seeds, offset=2 * n)[0])


@pytest.mark.parametrize("n", [131_072, 131_073])
def test_party_functions_small_call_boundary_bit_exact(n):
    """The per-party drop-in steps on both sides of SMALL_CALL_BYTES:
    party.mask_payload's masked vector and party.sum_decode's result
    bit-exact vs the oracle, the masker advanced by n."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.security.aggregation import party as P

    names = ["alice", "bob"]
    seeds = o.seeds_for(names)
    ms = [P.agree(P.new_masker(nm), {p: 0 for p in names}, {p: seeds[nm][p] for p in names if p != nm})
          for nm in names]
    rng = np.random.default_rng(n)
    xs = [(rng.standard_normal(n) * 0.1).astype(np.float32) for _ in names]
    masked = o.secure_masked(xs, names, seeds=seeds)
    pays = []
    for i, (m, x) in enumerate(zip(ms, xs)):
        pay, m2 = P.mask_payload(m, x, None, 0)
        assert np.array_equal(pay.u64, masked[i])
        assert m2.position(names[1 - i]) == n and m.position(names[1 - i]) == 0
        pays.append(pay)
    got = P.sum_decode(*pays, gpu=0)
    assert np.array_equal(got, o.secure_sum(xs, names, seeds=seeds)[0])


@pytest.mark.parametrize("parties,dtype", [(9, np.float64), (9, np.int64), (10, np.int64), (9, np.float32),
                                           (2, np.float32)])
def test_small_call_party_counts_containers_and_weights(parties, dtype):
    """The blocking small-call entries at their party limits (float32 fused:
    2..8, other types: 2..9; beyond them the general path), a tuple of
    layers, numpy-scalar weights for the average: bit-exact vs the oracle,
    round after round."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.device import PYU, reveal as rv
    from sfl_amd.security.aggregation import SecureAggregator

    names = [f"p{i:02d}" for i in range(parties)]
    seeds = o.seeds_for(names)
    pyus = [PYU(nm, 0) for nm in names]
    agg = SecureAggregator(PYU("server", 0), pyus,
                           seeds={(a, b): seeds[a][b] for a in names for b in names if a < b})
    rng = np.random.default_rng(parties)
    shapes = [(3, 5), (7,)]
    mk = (lambda sh: rng.integers(-500, 500, sh)) if dtype == np.int64 else \
        (lambda sh: rng.standard_normal(sh).astype(dtype))
    off = 0
    for rnd in range(2):
        layers = [tuple(mk(sh) for sh in shapes) for _ in names]
        objs = [p(lambda t=t: t)() for p, t in zip(pyus, layers)]
        got = rv(agg.sum(objs, axis=0))
        assert isinstance(got, tuple) and [g.shape for g in got] == shapes
        flat = [np.concatenate([a.reshape(-1) for a in t]) for t in layers]
        exp = o.secure_sum(flat, names, seeds=seeds, offset=off)[0]
        assert np.array_equal(np.concatenate([g.reshape(-1) for g in got]), exp), rnd
        off += 22
        ws = [np.int64(i + 1) if dtype == np.int64 else np.float32(0.5 * (i + 1)) for i in range(parties)]
        got = rv(agg.average(objs, axis=0, weights=ws))
        exp = o.secure_average(flat, names, weights=ws, seeds=seeds, offset=off)[0]
        assert np.array_equal(np.concatenate([g.reshape(-1) for g in got]), exp), rnd
        off += 22


@pytest.mark.parametrize("dtype", [np.int64, np.float64])
def test_general_one_call_matches_general_path(dtype, monkeypatch):
    """small float64 / int64 host calls of 2..9 parties take ONE
    blocking library call (``_host_general_one_call`` -> sa_clients_host).
    The same two rounds with that path forced off (the general per-launch
    path) give identical results, identical per-party digests and identical
    masker positions afterwards; both equal the oracle (digests of the
    oracle's masked vectors, decoded averages)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.device import PYU, reveal as rv
    from sfl_amd.security.aggregation import SecureAggregator

    names = ["alice", "bob", "carol", "dave"]
    seeds = o.seeds_for(names)
    pair = {(a, b): seeds[a][b] for a in names for b in names if a != b}
    pyus = [PYU(nm, 0) for nm in names]
    rng = np.random.default_rng(11)

    def layers():
        if dtype == np.int64:
            return [rng.integers(-1000, 1000, (3, 5)).astype(np.int64), rng.integers(-9, 9, 7).astype(np.int64)]
        return [rng.standard_normal((3, 5)), rng.standard_normal(7)]

    rounds = [[layers() for _ in names] for _ in range(2)]
    weights = [3, 1, 4, 2] if dtype == np.int64 else [0.5, 1.25, 2.0, 0.75]

    def run(one_call: bool):
        agg = SecureAggregator(PYU("server", 0), pyus, seeds=pair)
        calls = []
        orig = agg._host_general_one_call

        def spy(*a, **k):
            r = orig(*a, **k) if one_call else None
            calls.append(r is not None)
            return r

        monkeypatch.setattr(agg, "_host_general_one_call", spy)
        outs = []
        for data in rounds:
            got = rv(agg.average([p(lambda d=d: d)() for p, d in zip(pyus, data)], axis=0, weights=weights))
            digs = [np.asarray(d.cpu() if hasattr(d, "cpu") else d).view(np.uint64).copy()
                    for d in agg.last_digests if d is not None]
            outs.append((got, digs))
        pos = {nm: {p: agg._maskers[nm].position(p) for p in names if p != nm} for nm in names}
        return outs, pos, calls

    a, pos_a, calls_a = run(True)
    b, pos_b, calls_b = run(False)
    assert calls_a == [True, True] and calls_b == [False, False]
    assert pos_a == pos_b
    n = 22
    assert all(v == 2 * n for d in pos_a.values() for v in d.values())
    for r, ((ga, da), (gb, db)) in enumerate(zip(a, b)):
        for la, lb in zip(ga, gb):
            assert la.dtype == lb.dtype and np.array_equal(la, lb), r
        flat = [np.concatenate([x.reshape(-1) for x in d]) for d in rounds[r]]
        exp_avg, _, masked = o.secure_average(flat, names, weights=weights, seeds=seeds, offset=r * n)
        assert np.array_equal(np.concatenate([x.reshape(-1) for x in ga]), exp_avg), r
        want = [o.digest(m) for m in masked]
        assert [int(x) for x in np.concatenate(da)] == want, r
        assert [int(x) for x in np.concatenate(db)] == want, r
