"""Horizontal-FL round with the secure aggregator swapped in (BASELINE config
4): reference ``MlpNet`` shape (4-50-50-3,
tests/ml/nn/fl/model_def.py:55-69), ``fed_avg_w``, 8 clients, synthetic
iris-like data, ``aggregate_freq=1`` as in
tests/ml/nn/fl/test_fl_model_torch.py:312-319.

CPU: the FL loop with the oracle aggregator learns (host logic).
GPU: the same loop with the HIP ``SecureAggregator`` gives, round after
round, aggregated parameters bit-identical to the oracle's, hence identical
final models (local training runs on the CPU in both, so it is
deterministic)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
from torch import nn  # noqa: E402
from torch.nn import functional as F  # noqa: E402

from oracle import secagg as o  # noqa: E402

NAMES = [f"client{i}" for i in range(8)]


class MlpNet(nn.Module):
    def __init__(self):
        super().__init__()
        self.layer1 = nn.Linear(4, 50)
        self.layer2 = nn.Linear(50, 50)
        self.layer3 = nn.Linear(50, 3)

    def forward(self, x):
        x = F.relu(self.layer1(x))
        x = F.relu(self.layer2(x))
        return self.layer3(x)


def _data(n_per=96, seed=0):
    rng = np.random.default_rng(seed)
    centers = np.array([[0, 0, 0, 0], [2, 2, 0, 1], [0, 2, 2, -1]], dtype=np.float32)
    xs, ys = [], []
    for _ in NAMES:
        y = rng.integers(0, 3, n_per)
        x = centers[y] + rng.standard_normal((n_per, 4)).astype(np.float32) * 0.6
        xs.append(x.astype(np.float32))
        ys.append(y.astype(np.int64))
    return xs, ys


class OracleAggregator:
    """Test-only Aggregator on the CPU oracle (numpy restatement): per-layer
    secure average with the stream offset advancing layer by layer."""

    def __init__(self, names, seeds):
        self.names, self.seeds, self.offset = names, seeds, 0

    def average(self, data, axis=0, weights=None):
        from sfl_amd.device import PYUObject

        payloads = [d.data for d in data]
        out = []
        for li in range(len(payloads[0])):
            xs = [np.asarray(p[li]) for p in payloads]
            avg, _, _ = o.secure_average(xs, self.names, weights=weights, seeds=self.seeds, offset=self.offset)
            self.offset += xs[0].size
            out.append(avg.reshape(xs[0].shape))
        return PYUObject(data[0].device, out)


def _fl(aggregator, pyus, epochs=3, hook=None, dp_strategy=None):
    from torch import optim

    from sfl_amd.ml.fl import FLModel, TorchModel, optim_wrapper

    model = TorchModel(model_fn=MlpNet, loss_fn=nn.CrossEntropyLoss, optim_fn=optim_wrapper(optim.Adam, lr=5e-3))
    fl = FLModel(server=None, device_list=pyus, model=model, aggregator=aggregator, strategy="fed_avg_w",
                 backend="torch", random_seed=1234, train_device="cpu", dp_strategy=dp_strategy)
    xs, ys = _data()
    hist = fl.fit({p: x for p, x in zip(pyus, xs)}, {p: y for p, y in zip(pyus, ys)}, batch_size=32, epochs=epochs,
                  aggregate_freq=1, validation_data=(np.concatenate(xs), np.concatenate(ys)), round_hook=hook)
    return fl, hist


def test_fl_round_with_oracle_aggregator_learns():
    from sfl_amd.device import PYU

    pyus = [PYU(n, None) for n in NAMES]
    fl, hist = _fl(OracleAggregator(NAMES, o.seeds_for(NAMES)), pyus, epochs=4)
    assert hist["val_accuracy"][-1] > 0.8
    assert hist["train_loss"][-1] < hist["train_loss"][0]
    # every party ends with the aggregated model
    w0 = fl.get_weights(pyus[0])
    for p in pyus[1:]:
        assert all(np.array_equal(a, b) for a, b in zip(w0, fl.get_weights(p)))


def test_fit_averages_initial_weights_first():
    """Reference fit (fl_model.py:473 -> :126-138): the first aggregation is
    the unweighted average of every worker's initial weights, installed on
    every worker before the first round; later rounds are weighted by the
    sample counts (:516-518)."""
    from sfl_amd.device import PYU

    class Recording(OracleAggregator):
        def __init__(self, *a):
            super().__init__(*a)
            self.calls = []

        def average(self, data, axis=0, weights=None):
            self.calls.append((weights, [[np.array(a) for a in d.data] for d in data]))
            return super().average(data, axis=axis, weights=weights)

    pyus = [PYU(n, None) for n in NAMES]
    agg = Recording(NAMES, o.seeds_for(NAMES))
    hooks = []
    _fl(agg, pyus, epochs=1, hook=lambda r, p: hooks.append(r))
    assert hooks == [-1, 0, 1, 2]
    assert len(agg.calls) == 4
    w0, init_payloads = agg.calls[0]
    assert w0 is None
    # every worker was seeded alike (fl_base.py:51-52): identical initial weights
    for p in init_payloads[1:]:
        assert all(np.array_equal(a, b) for a, b in zip(init_payloads[0], p))
    assert all(w == [32] * 8 for w, _ in agg.calls[1:])  # per-round sample counts (batch 32)
    # the first round's global weights are the decoded init average (a 2^-18 grid), not the raw init
    first_round_inputs = agg.calls[1][1]
    assert not all(np.array_equal(a, b) for a, b in zip(init_payloads[0], first_round_inputs[0]))


@pytest.mark.gpu
def test_fl_round_hip_aggregator_bit_exact_vs_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.device import PYU
    from sfl_amd.security.aggregation import SecureAggregator

    seeds = o.seeds_for(NAMES)
    pair = {(a, b): seeds[a][b] for a in NAMES for b in NAMES if a != b}
    pyus = [PYU(n, 0) for n in NAMES]
    ref_rounds, hip_rounds = [], []
    fl_ref, h_ref = _fl(OracleAggregator(NAMES, seeds), pyus, hook=lambda r, p: ref_rounds.append(p))
    agg = SecureAggregator(PYU("server", 0), pyus, seeds=pair)
    fl_hip, h_hip = _fl(agg, pyus, hook=lambda r, p: hip_rounds.append(p))
    assert len(ref_rounds) == len(hip_rounds) == 1 + 3 * 3  # init average + rounds
    for r, (a, b) in enumerate(zip(ref_rounds, hip_rounds)):
        for li, (x, y) in enumerate(zip(a, b)):
            assert x.dtype == y.dtype == np.float64
            assert np.array_equal(x, y), (r, li)
    for x, y in zip(fl_ref.get_weights(), fl_hip.get_weights()):
        assert np.array_equal(x, y)
    assert h_ref["val_accuracy"] == h_hip["val_accuracy"]


@pytest.mark.gpu
def test_fl_round_with_gaussian_dp_hip_vs_oracle_aggregator():
    """DPStrategyFL(GaussianModelDP) on the clients (fed_avg_w.py:80-85), same
    keyed noise in both runs: the HIP aggregator's rounds equal the oracle's."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.device import PYU
    from sfl_amd.security.aggregation import SecureAggregator
    from sfl_amd.security.privacy import DPStrategyFL, GaussianModelDP

    seeds = o.seeds_for(NAMES)
    pair = {(a, b): seeds[a][b] for a in NAMES for b in NAMES if a != b}
    pyus = [PYU(n, 0) for n in NAMES]
    mk = lambda: DPStrategyFL(GaussianModelDP(noise_multiplier=0.05, num_clients=8, l2_norm_clip=5.0,  # noqa: E731
                                              seed=2024))
    ref_rounds, hip_rounds = [], []
    _fl(OracleAggregator(NAMES, seeds), pyus, epochs=1, hook=lambda r, p: ref_rounds.append(p), dp_strategy=mk())
    agg = SecureAggregator(PYU("server", 0), pyus, seeds=pair)
    _, h = _fl(agg, pyus, epochs=1, hook=lambda r, p: hip_rounds.append(p), dp_strategy=mk())
    assert len(ref_rounds) == len(hip_rounds) == 1 + 3
    for a, b in zip(ref_rounds, hip_rounds):
        for x, y in zip(a, b):
            assert np.array_equal(x, y)


@pytest.mark.gpu
def test_fl_round_through_the_per_party_drop_in_bit_exact_vs_oracle():
    """BASELINE config 4 with the secretflow-facing drop-in
    (sfl_amd.compat.secretflow: every party masks on its own device through
    party.mask_payload, only masked payloads reach the server) as the FLModel
    aggregator: init average and every round equal the oracle's bit for bit."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.compat import secretflow as hip
    from sfl_amd.device import PYU

    seeds = o.seeds_for(NAMES)
    pair = {(a, b): seeds[a][b] for a in NAMES for b in NAMES if a != b}
    pyus = [PYU(n, 0) for n in NAMES]
    ref_rounds, hip_rounds = [], []
    _fl(OracleAggregator(NAMES, seeds), pyus, epochs=2, hook=lambda r, p: ref_rounds.append(p))
    agg = hip.SecureAggregator(PYU("server", 0), pyus, seeds=pair)
    _fl(agg, pyus, epochs=2, hook=lambda r, p: hip_rounds.append(p))
    assert len(ref_rounds) == len(hip_rounds) == 1 + 2 * 3
    for r, (a, b) in enumerate(zip(ref_rounds, hip_rounds)):
        for li, (x, y) in enumerate(zip(a, b)):
            assert np.array_equal(x, y), (r, li)
