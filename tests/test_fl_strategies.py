"""The other FL payload producers of SURVEY.md §8(a8) with the secure
aggregator swapped in: ``fed_avg_u`` (clients upload model updates,
fed_avg_u.py:30-96) and ``fed_avg_g`` (clients upload gradients,
fed_avg_g.py:28-112).  Same setup as tests/test_fl_round.py (reference
MlpNet 4-50-50-3, 8 clients, synthetic iris-like data, aggregate_freq=1).

CPU: with the oracle aggregator both strategies train (and with fed_avg_g
every party ends with the same model).  GPU: with the HIP ``SecureAggregator`` every round's
aggregate (small signed updates / gradients) equals the oracle's bit for
bit, and so do the final models."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
from torch import nn  # noqa: E402

from oracle import secagg as o  # noqa: E402
from test_fl_round import NAMES, MlpNet, OracleAggregator, _data  # noqa: E402

STRATEGIES = ["fed_avg_u", "fed_avg_g"]


def _fl(strategy, aggregator, pyus, epochs=3, hook=None, aggregate_freq=1):
    from torch import optim

    from sfl_amd.ml.fl import FLModel, TorchModel, optim_wrapper

    lr = 5e-3 if strategy == "fed_avg_u" else 2e-2
    model = TorchModel(model_fn=MlpNet, loss_fn=nn.CrossEntropyLoss, optim_fn=optim_wrapper(optim.Adam, lr=lr))
    fl = FLModel(server=None, device_list=pyus, model=model, aggregator=aggregator, strategy=strategy,
                 backend="torch", random_seed=1234, train_device="cpu")
    xs, ys = _data()
    hist = fl.fit({p: x for p, x in zip(pyus, xs)}, {p: y for p, y in zip(pyus, ys)}, batch_size=32, epochs=epochs,
                  aggregate_freq=aggregate_freq, validation_data=(np.concatenate(xs), np.concatenate(ys)),
                  round_hook=hook)
    return fl, hist


@pytest.mark.parametrize("strategy", STRATEGIES)
def test_strategy_with_oracle_aggregator_learns(strategy):
    from sfl_amd.device import PYU

    pyus = [PYU(n, None) for n in NAMES]
    rounds = []
    fl, hist = _fl(strategy, OracleAggregator(NAMES, o.seeds_for(NAMES)), pyus, epochs=4,
                   hook=lambda r, p: rounds.append(p))
    assert hist["val_accuracy"][-1] > 0.7, hist["val_accuracy"]
    # the aggregated payloads are signed deltas / gradients, not weights
    assert any((a < 0).any() for a in rounds[-1])
    if strategy == "fed_avg_g":  # only the aggregated gradients move the models
        w0 = fl.get_weights(pyus[0])
        for p in pyus[1:]:
            assert all(np.array_equal(a, b) for a, b in zip(w0, fl.get_weights(p)))
    # fed_avg_u: each party adds the averaged update to its OWN locally trained
    # weights (fed_avg_u.py:55-57, :86-95), so the parties' models differ


@pytest.mark.gpu
@pytest.mark.parametrize("strategy", STRATEGIES)
def test_strategy_hip_aggregator_bit_exact_vs_oracle(strategy):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.device import PYU
    from sfl_amd.security.aggregation import SecureAggregator

    seeds = o.seeds_for(NAMES)
    pair = {(a, b): seeds[a][b] for a in NAMES for b in NAMES if a != b}
    pyus = [PYU(n, 0) for n in NAMES]
    ref_rounds, hip_rounds = [], []
    fl_ref, h_ref = _fl(strategy, OracleAggregator(NAMES, seeds), pyus, hook=lambda r, p: ref_rounds.append(p))
    agg = SecureAggregator(PYU("server", 0), pyus, seeds=pair)
    fl_hip, h_hip = _fl(strategy, agg, pyus, hook=lambda r, p: hip_rounds.append(p))
    assert len(ref_rounds) == len(hip_rounds) == 1 + 9  # init average + rounds
    for r, (a, b) in enumerate(zip(ref_rounds, hip_rounds)):
        for li, (x, y) in enumerate(zip(a, b)):
            assert np.array_equal(x, y), (r, li)
    for x, y in zip(fl_ref.get_weights(), fl_hip.get_weights()):
        assert np.array_equal(x, y)
    assert h_ref["val_accuracy"] == h_hip["val_accuracy"]


def test_fed_avg_g_concatenates_step_gradients_like_the_reference():
    """fed_avg_g.py:91 ``local_gradients_sum += local_gradients`` on lists:
    with aggregate_freq = 2 (the reference's own fed_avg_g test,
    tests/ml/nn/fl/test_fl_model_torch.py:81) the aggregated payload holds
    2 x the parameter arrays; the models step with the first half."""
    from sfl_amd.device import PYU

    pyus = [PYU(n, None) for n in NAMES]
    rounds = []
    _fl("fed_avg_g", OracleAggregator(NAMES, o.seeds_for(NAMES)), pyus, epochs=1, hook=lambda r, p: rounds.append(p),
        aggregate_freq=2)
    n_params = len(list(MlpNet().parameters()))
    # rounds[0] is the init average of the 6 weight arrays; then 3 steps / 2 -> rounds of 2 steps and 1 step
    assert len(rounds[1]) == 2 * n_params and len(rounds[2]) == n_params
    assert [a.shape for a in rounds[1][:n_params]] == [a.shape for a in rounds[1][n_params:]]


@pytest.mark.gpu
def test_fed_avg_g_aggregate_freq_2_hip_bit_exact_vs_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.device import PYU
    from sfl_amd.security.aggregation import SecureAggregator

    seeds = o.seeds_for(NAMES)
    pair = {(a, b): seeds[a][b] for a in NAMES for b in NAMES if a != b}
    pyus = [PYU(n, 0) for n in NAMES]
    ref_rounds, hip_rounds = [], []
    fl_ref, _ = _fl("fed_avg_g", OracleAggregator(NAMES, seeds), pyus, epochs=2,
                    hook=lambda r, p: ref_rounds.append(p), aggregate_freq=2)
    agg = SecureAggregator(PYU("server", 0), pyus, seeds=pair)
    fl_hip, _ = _fl("fed_avg_g", agg, pyus, epochs=2, hook=lambda r, p: hip_rounds.append(p), aggregate_freq=2)
    assert len(ref_rounds) == len(hip_rounds) == 1 + 2 * 2
    for a, b in zip(ref_rounds, hip_rounds):
        assert len(a) == len(b)
        for x, y in zip(a, b):
            assert np.array_equal(x, y)
    for x, y in zip(fl_ref.get_weights(), fl_hip.get_weights()):
        assert np.array_equal(x, y)
