"""MOON end-to-end with the secure aggregator swapped in (SURVEY.md §8f row
1), following the reference's tests/ml/nn/fl/strategy/test_moon_torch.py:
the same ConvNet (conv head + projection MLP + classifier, :27-65),
``strategy="moon"``, ``model_buffer_size=1``, two parties holding 0.4 / 0.6
of the data, ``epochs=1, batch_size=32, aggregate_freq=1`` (:93-125), then
``predict`` sizes and ``evaluate`` == the last validation accuracy
(:127-149).  MNIST is not available offline: the data are synthetic 28x28
images of 10 noisy class prototypes (1000 rows instead of 10000).

CPU: the loop with the oracle aggregator trains (host logic).
GPU: with the HIP ``SecureAggregator`` every round's aggregated parameters
equal the oracle aggregator's bit for bit (local training on the CPU in
both runs, so it is deterministic)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
from torch import nn  # noqa: E402
from torch.nn import functional as F  # noqa: E402

from oracle import secagg as o  # noqa: E402
from test_fl_round import OracleAggregator  # noqa: E402

NAMES = ["alice", "bob"]


class ConvNet(nn.Module):
    """The reference test's ConvNet (test_moon_torch.py:27-65)."""

    def __init__(self, cosine_similarity_fn, out_dim=256, temperature=0.5, mu=1):
        super().__init__()
        self.cosine_similarity_fn = cosine_similarity_fn
        self.out_dim = out_dim
        self.temperature = temperature
        self.mu = mu
        self.head = nn.Sequential(
            nn.Conv2d(1, 3, kernel_size=3),
            nn.MaxPool2d(kernel_size=3),
            nn.ReLU(),
            nn.Flatten(),
            nn.Linear(192, 128),
            nn.ReLU(),
            nn.Linear(128, 64),
        )
        self.l1 = nn.Linear(64, 64)
        self.l2 = nn.Linear(64, self.out_dim)
        self.l3 = nn.Linear(self.out_dim, 10)

    def forward(self, x, return_all=False):
        h = self.head(x).squeeze()
        z = self.l2(F.relu(self.l1(h)))
        y = self.l3(z)
        return (h, z, y) if return_all else y


def _data(n=1000, seed=7):
    rng = np.random.default_rng(seed)
    protos = (rng.random((10, 1, 28, 28)) > 0.75).astype(np.float32)
    y = rng.integers(0, 10, n)
    x = protos[y] + rng.standard_normal((n, 1, 28, 28)).astype(np.float32) * 0.4
    cut = int(n * 0.4)
    return [x[:cut], x[cut:]], [y[:cut].astype(np.int64), y[cut:].astype(np.int64)]


def _moon(aggregator, pyus, hook=None):
    from torch import optim

    from sfl_amd.ml.fl import FLModel, TorchModel, optim_wrapper

    model = TorchModel(model_fn=ConvNet, loss_fn=nn.CrossEntropyLoss, optim_fn=optim_wrapper(optim.Adam, lr=1e-2),
                       cosine_similarity_fn=nn.CosineSimilarity(dim=-1))
    fl = FLModel(server=None, device_list=pyus, model=model, aggregator=aggregator, strategy="moon",
                 backend="torch", random_seed=1234, train_device="cpu", model_buffer_size=1)
    xs, ys = _data()
    hist = fl.fit({p: x for p, x in zip(pyus, xs)}, {p: y for p, y in zip(pyus, ys)}, batch_size=32, epochs=1,
                  aggregate_freq=1, validation_data=(np.concatenate(xs), np.concatenate(ys)), round_hook=hook)
    return fl, hist, xs, ys


def test_moon_with_oracle_aggregator():
    from sfl_amd.device import PYU, reveal

    pyus = [PYU(n, None) for n in NAMES]
    fl, hist, xs, ys = _moon(OracleAggregator(NAMES, o.seeds_for(NAMES)), pyus)
    pred = fl.predict({p: x for p, x in zip(pyus, xs)}, batch_size=32)
    assert len(reveal(pred[pyus[0]])) == len(xs[0]) == 400
    _, acc = fl.evaluate(np.concatenate(xs), np.concatenate(ys))
    assert acc == hist["val_accuracy"][-1]
    assert acc > 0.1
    w0 = fl.get_weights(pyus[0])
    assert all(np.array_equal(a, b) for a, b in zip(w0, fl.get_weights(pyus[1])))


@pytest.mark.gpu
def test_moon_hip_aggregator_bit_exact_vs_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.device import PYU
    from sfl_amd.security.aggregation import SecureAggregator

    seeds = o.seeds_for(NAMES)
    pair = {(a, b): seeds[a][b] for a in NAMES for b in NAMES if a != b}
    pyus = [PYU(n, 0) for n in NAMES]
    ref_rounds, hip_rounds = [], []
    fl_ref, h_ref, _, _ = _moon(OracleAggregator(NAMES, seeds), pyus, hook=lambda r, p: ref_rounds.append(p))
    agg = SecureAggregator(PYU("server", 0), pyus, seeds=pair)
    fl_hip, h_hip, _, _ = _moon(agg, pyus, hook=lambda r, p: hip_rounds.append(p))
    assert len(ref_rounds) == len(hip_rounds) > 0
    for r, (a, b) in enumerate(zip(ref_rounds, hip_rounds)):
        for li, (x, y) in enumerate(zip(a, b)):
            assert np.array_equal(x, y), (r, li)
    for x, y in zip(fl_ref.get_weights(), fl_hip.get_weights()):
        assert np.array_equal(x, y)
    assert h_ref["val_accuracy"] == h_hip["val_accuracy"]
