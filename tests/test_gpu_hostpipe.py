"""sfl_amd/hostpipe.py's one-shot host copies on the GPU: ``d2h`` / ``h2d``
(no pageable DMA: pooled registered buffers or pinned staging) round-trip
every element type, shape and placement the product hands them, bit for
bit."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


CASES = [
    (np.float32, (3_000_001,)),  # 12 MB: a pooled result
    (np.float64, (1001, 997)),
    (np.int64, (2_000_003,)),
    (np.int32, (17,)),
    (np.float16, (4, 5, 6)),
    (np.bool_, (1000,)),
    (np.float64, ()),
    (np.float32, (0,)),
]


@pytest.mark.parametrize("pooled", [True, False])
@pytest.mark.parametrize("dt,shape", CASES)
def test_d2h_h2d_round_trip(dt, shape, pooled, monkeypatch):
    from sfl_amd import hostpipe as H

    monkeypatch.setattr(H, "RESULTS", H.ResultPool(1 << 30))
    rng = np.random.default_rng(7)
    a = (rng.standard_normal(shape) * 1e3).astype(dt) if dt != np.bool_ else rng.random(shape) < 0.5
    dev = torch.device("cuda", 0)
    t = H.h2d(a, dev)
    assert t.device == dev and tuple(t.shape) == shape
    back = H.d2h(t, pooled=pooled)
    assert back.dtype == np.dtype(dt) and back.shape == shape
    assert np.array_equal(back.reshape(-1).view(np.uint8), np.ascontiguousarray(a).reshape(-1).view(np.uint8))
    if pooled and a.nbytes >= 8 << 20:
        assert H.RESULTS.contains(back)  # straight into a registered buffer
    else:
        assert not H.RESULTS.contains(back)
    del back
    H.RESULTS.clear()


def test_d2h_h2d_views_tensors_and_u64(monkeypatch):
    from sfl_amd import hostpipe as H

    monkeypatch.setattr(H, "RESULTS", H.ResultPool(1 << 30))
    dev = torch.device("cuda", 0)
    base = torch.arange(4_000_000, dtype=torch.int64, device=dev).reshape(2000, 2000)
    view = base.t()[::2]  # non-contiguous device view
    assert np.array_equal(H.d2h(view), view.cpu().numpy())
    # uint64 host arrays (masked vectors) go up as their int64 bits
    u = np.arange(2**64 - 1000, 2**64 - 1, dtype=np.uint64)
    t = H.h2d(u, dev)
    assert t.dtype == torch.int64 and np.array_equal(H.d2h(t).view(np.uint64), u)
    # a CPU tensor is a host array; a device tensor is moved as it is
    x = torch.randn(300_001)
    assert torch.equal(H.h2d(x, dev).cpu(), x)
    y = torch.randn(10, device=dev)
    assert H.h2d(y, dev).data_ptr() == y.data_ptr()
    # an array inside a pooled result is copied as it is (already registered)
    owner = H.RESULTS.take(16 << 20)
    pooled = owner[: 8 << 20].view(np.float64)
    pooled[:] = np.arange(pooled.size)
    assert torch.equal(H.h2d(pooled[5:], dev).cpu(), torch.from_numpy(pooled[5:]))
    with pytest.raises(TypeError, match="no host array type"):
        H.d2h(torch.zeros(3, dtype=torch.bfloat16, device=dev))
    del owner, pooled
    H.RESULTS.clear()


def test_gpu_model_weights_round_trip_without_pageable_copies():
    """FedAvgW on a GPU model: get_weights (hostpipe.d2h) and set_weights
    from numpy arrays, CPU tensors and device tensors (hostpipe.h2d or a
    device copy) give back the same bits; a float64 array loads into the
    float32 parameters as the reference's torch.Tensor(np.copy(v)) does."""
    from torch import nn, optim

    from sfl_amd.device import PYU
    from sfl_amd.ml.fl import FedAvgW, TorchModel, optim_wrapper

    class Net(nn.Module):
        def __init__(self):
            super().__init__()
            self.a = nn.Linear(1000, 3000)  # 12 MB of weights: a pooled-size array
            self.b = nn.Linear(3000, 7)

    torch.manual_seed(0)
    m = TorchModel(model_fn=Net, loss_fn=nn.CrossEntropyLoss, optim_fn=optim_wrapper(optim.SGD, lr=0.1))
    w = FedAvgW(m, PYU("alice", 0))
    assert next(w.model.parameters()).is_cuda
    ws = w.get_weights()
    assert [a.dtype for a in ws] == [np.float32] * 4
    ref = [p.detach().cpu().numpy().copy() for p in w.model.state_dict().values()]
    assert all(np.array_equal(a, r) for a, r in zip(ws, ref))
    for form in ("numpy", "cpu", "cuda", "f64"):
        new = [np.asarray(a) * 2 + 1 for a in ws]
        give = {"numpy": new, "cpu": [torch.from_numpy(a) for a in new],
                "cuda": [torch.from_numpy(a).cuda() for a in new],
                "f64": [a.astype(np.float64) for a in new]}[form]
        w.set_weights(give)
        got = w.get_weights()
        assert all(np.array_equal(g, a.astype(np.float32)) for g, a in zip(got, new)), form
        td = w.get_weights(return_numpy=False)
        assert all(t.device.type == "cpu" and np.array_equal(t.numpy(), g) for t, g in zip(td.values(), got)), form
