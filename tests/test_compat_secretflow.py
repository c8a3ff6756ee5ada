"""The secretflow-shaped import path (sfl_amd.compat.secretflow): duck-typed
stand-ins for secretflow's PYU / PYUObject / sf.reveal, as the reference's
callers hand them to ``SecureAggregator(device, participants, fxp_bits)``.

CPU: device mapping, ``install`` rebinding, argument checks.  GPU: the
AggregatorBase-style sums / averages through the adapter equal the oracle's
bit for bit, weights given as device objects on the client parties
(stateful_fedgen_aggregator.py:74-78)."""
import types

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import secagg as o  # noqa: E402


class FakePYU:
    """secretflow.PYU shape: .party, __call__(fn) -> fn run 'on' the party."""

    def __init__(self, party):
        self.party = party

    def __call__(self, fn):
        return lambda *a: FakeObj(self, fn(*a))

    def __repr__(self):
        return f"FakePYU({self.party})"


class FakeObj:
    """secretflow.PYUObject shape: .device and an opaque reference."""

    def __init__(self, device, value):
        self.device = device
        self._ref = {"value": value}


def fake_reveal(obj):
    return obj._ref["value"]


def test_adapter_maps_devices_and_installs():
    from sfl_amd.compat import secretflow as hip

    alice, bob, carol = FakePYU("alice"), FakePYU("bob"), FakePYU("carol")
    agg = hip.SecureAggregator(carol, [alice, bob], reveal=fake_reveal, gpu_of={"alice": 0, "bob": 0, "carol": 0}.get)
    assert agg.device is carol and agg.participants == [alice, bob]
    assert [p.party for p in agg.inner.participants] == ["alice", "bob"]
    assert agg.inner.device.party == "carol"
    m = types.ModuleType("secretflow_security_aggregation")
    hip.install(m)
    assert m.SecureAggregator is hip.SecureAggregator
    with pytest.raises(TypeError):
        hip.SecureAggregator(object(), [alice])
    with pytest.raises(AssertionError, match="empty"):
        agg.sum([], axis=0)
    with pytest.raises(AssertionError, match="not a participant"):
        agg.sum([FakeObj(FakePYU("mallory"), np.zeros(3))], axis=0)
    # a device-object weight on another party than its data is refused before
    # anything is revealed (stateful_fedgen_aggregator.py:74-78)
    data = [alice(lambda: np.ones(3))(), bob(lambda: np.ones(3))()]
    with pytest.raises(AssertionError, match="Device of weight does not match"):
        agg.average(data, axis=0, weights=[bob(lambda: 1)(), bob(lambda: 2)()])
    with pytest.raises(AssertionError, match="Length of the weights"):
        agg.average(data, axis=0, weights=[1])


@pytest.mark.gpu
def test_adapter_aggregates_like_the_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.compat import secretflow as hip

    names = ["alice", "bob", "carol"]
    seeds = o.seeds_for(names)
    pair = {(a, b): seeds[a][b] for a in names for b in names if a != b}
    devs = [FakePYU(n) for n in names]
    server = FakePYU("server")
    agg = hip.SecureAggregator(server, devs, reveal=fake_reveal, seeds=pair)
    rng = np.random.default_rng(5)
    xs = [(rng.standard_normal((4, 6)) * 0.1).astype(np.float32) for _ in names]
    objs = [d(lambda x=x: x)() for d, x in zip(devs, xs)]
    s = agg.sum(objs, axis=0)
    assert isinstance(s, FakeObj) and s.device is server
    exp, _, _ = o.secure_sum([x.reshape(-1) for x in xs], names, seeds=seeds)
    assert np.array_equal(fake_reveal(s).reshape(-1), exp)
    w = [d(lambda k=k: 10 * (k + 1))() for k, d in enumerate(devs)]  # weights on the clients' devices
    avg = agg.average(objs, axis=0, weights=w)
    exp, _, _ = o.secure_average([x.reshape(-1) for x in xs], names, weights=[10, 20, 30], seeds=seeds,
                                 offset=xs[0].size)
    assert np.array_equal(fake_reveal(avg).reshape(-1), exp)
