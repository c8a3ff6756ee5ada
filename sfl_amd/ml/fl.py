"""Horizontal-FL round around the secure aggregator (SURVEY.md §8f row 1,
BASELINE config 4): the caller side of the hot path, mirrored from the
reference so the aggregator can be swapped in exactly where FLModel uses it.

Reference interfaces followed:

* ``FLModel.fit`` aggregation hooks -- the initial weights of every worker
  are averaged through the aggregator and installed everywhere before the
  first epoch (``fl_model.py:473`` -> ``initialize_weights``, ``:126-138``);
  every ``aggregate_freq`` local steps the
  clients' ``train_step`` outputs go to ``aggregator.average(params, axis=0,
  weights=sample_nums)`` and the result is sent back to every party
  (``sfl/ml/nn/fl/fl_model.py:492-517``, ``:578-583``); the last batch of an
  epoch is applied with ``apply_weights`` (``:585-589``);
* ``FedAvgW.train_step`` -- set the global weights, run ``train_steps``
  batches, return ``(get_weights(return_numpy=True), num_sample)``
  (``sfl/ml/nn/fl/backend/torch/strategy/fed_avg_w.py:36-87``);
* torch payload packing -- ``state_dict`` values as a list of host numpy
  arrays, written back with ``torch.Tensor(np.copy(v))``
  (``sfl/ml/nn/core/torch/mixins.py:74-89``);
* ``TorchModel(model_fn, loss_fn, optim_fn, metrics)`` and ``optim_wrapper``
  (``sfl/ml/nn/core/torch/module.py:247``, ``sfl/ml/nn/core/torch/utils.py:23``);
  each worker seeds torch with ``random_seed`` before building its model
  (``sfl/ml/nn/fl/backend/torch/fl_base.py:51-52``), so every client starts
  from the same initial weights.

Parties are ``PYU``s (``sfl_amd.device``); local training runs on
``train_device`` (the party's GPU by default, or the CPU).  Out of scope:
the reference's dataset builders, callbacks, DP accountant hooks,
compression strategies and the other strategies (fed_prox, scaffold, ...);
``moon`` is mirrored because its reference test is the FL end-to-end the
survey names for the aggregator swap, ``fed_avg_u``
and ``fed_avg_g`` because they are the other payload producers of §8(a8)
(model updates and gradients instead of weights).
"""

from __future__ import annotations

import copy
import math
import time
from typing import Callable, Dict, List, Optional

import numpy as np
import torch

from .. import hostpipe as H
from ..device import PYU, PYUObject, reveal


def _host_array(v: torch.Tensor) -> np.ndarray:
    """A fresh host copy of a model tensor (``.cpu().numpy().copy()``): a GPU
    tensor's through pinned memory, never a pageable DMA (``hostpipe.d2h``:
    the aggregator in the same process keeps registered host buffers)."""
    v = v.detach()
    return v.numpy().copy() if v.device.type == "cpu" else H.d2h(v, pooled=False)


def _host_tensor(v: torch.Tensor) -> torch.Tensor:
    """``v.cpu()`` the same way (element types numpy lacks keep ``.cpu()``)."""
    if v.device.type == "cpu" or H.host_dtype(v) is None:
        return v.cpu()
    return torch.from_numpy(H.d2h(v, pooled=False))


def optim_wrapper(func, *args, **kwargs):
    """``optim_wrapper(optim.Adam, lr=1e-2)(params)`` (reference utils.py:23)."""

    def make(params):
        return func(params, *args, **kwargs)

    return make


class TorchModel:
    """Model builder record (reference module.py:247): extra keyword
    arguments go to ``model_fn`` (e.g. MOON's ``cosine_similarity_fn``,
    tests/ml/nn/fl/strategy/test_moon_torch.py:76-91)."""

    def __init__(self, model_fn: Callable[..., torch.nn.Module] = None, loss_fn: Callable = None,
                 optim_fn: Callable = None, metrics: Optional[list] = None, **kwargs):
        self.model_fn = model_fn
        self.loss_fn = loss_fn
        self.optim_fn = optim_fn
        self.metrics = list(metrics or [])
        self.kwargs = kwargs


class FedAvgW:
    """One party's worker for the ``fed_avg_w`` strategy."""

    def __init__(self, builder: TorchModel, device: PYU, random_seed: Optional[int] = None,
                 train_device: Optional[torch.device] = None, **kwargs):
        if random_seed is not None:
            torch.manual_seed(random_seed)
        self.device = device
        self.exe_device = torch.device(train_device) if train_device is not None else device.torch_device
        self.model = builder.model_fn(**builder.kwargs).to(self.exe_device)
        self.optimizer = builder.optim_fn(self.model.parameters())
        self.loss_fn = builder.loss_fn()
        self._x = self._y = None
        self._batch = 32
        self._pos = 0

    # ----------------------------------------------------------- data
    def set_data(self, x: np.ndarray, y: np.ndarray, batch_size: int):
        self._x = torch.as_tensor(np.asarray(x, dtype=np.float32))
        self._y = torch.as_tensor(np.asarray(y))
        self._batch = int(batch_size)
        self._pos = 0

    def steps_per_epoch(self) -> int:
        return math.ceil(len(self._x) / self._batch)

    def _reset_data_iter(self):
        self._pos = 0

    def next_batch(self):
        if self._pos >= len(self._x):
            self._pos = 0
        lo, hi = self._pos, min(len(self._x), self._pos + self._batch)
        self._pos = hi
        return self._x[lo:hi].to(self.exe_device), self._y[lo:hi].to(self.exe_device)

    # -------------------------------------------------------- weights
    def get_weights(self, return_numpy: bool = True):
        if not return_numpy:
            return {k: _host_tensor(v) for k, v in self.model.state_dict().items()}
        return [_host_array(v) for v in self.model.state_dict().values()]

    def set_weights(self, weights, model: Optional[torch.nn.Module] = None):
        model = self.model if model is None else model
        sd = model.state_dict()
        new = {}
        for (k, v), w in zip(sd.items(), weights):
            if v.device.type != "cpu":
                # a GPU model: the weights reach its device by a pinned copy
                # (hostpipe.h2d, never a pageable DMA) or device to device, so
                # load_state_dict copies on the device
                t = w.detach().to(v.device) if isinstance(w, torch.Tensor) and w.device.type != "cpu" else \
                    H.h2d(w.detach() if isinstance(w, torch.Tensor) else np.asarray(w), v.device)
                new[k] = t.to(dtype=v.dtype)
                continue
            # reference: torch.Tensor(np.copy(v)) -> float32 for float params
            w = _host_array(w) if isinstance(w, torch.Tensor) else np.array(w, copy=True)
            new[k] = torch.from_numpy(w).to(dtype=v.dtype)
        model.load_state_dict(new)

    # ------------------------------------------------------- training
    def train_step(self, weights, cur_steps: int, train_steps: int, refresh_data: bool = False,
                   dp_strategy=None, **kwargs):
        self.model.train()
        if refresh_data:
            self._reset_data_iter()
        if weights is not None:
            self.set_weights(weights)
        num_sample = 0
        loss = None
        for _ in range(train_steps):
            x, y = self.next_batch()
            num_sample += x.shape[0]
            self.optimizer.zero_grad()
            loss = self.loss_fn(self.model(x), y)
            loss.backward()
            self.optimizer.step()
        self.last_loss = float(loss.item()) if loss is not None else float("nan")
        model_weights = self.get_weights(return_numpy=True)
        if dp_strategy is not None and dp_strategy.model_gdp is not None:  # fed_avg_w.py:80-85
            model_weights = dp_strategy.model_gdp(model_weights)
        return model_weights, num_sample

    def apply_weights(self, weights, **kwargs):
        if weights is not None:
            self.set_weights(weights)

    @torch.no_grad()
    def evaluate(self, x, y):
        self.model.eval()
        xt = torch.as_tensor(np.asarray(x, dtype=np.float32)).to(self.exe_device)
        yt = torch.as_tensor(np.asarray(y)).to(self.exe_device)
        out = self.model(xt)
        loss = float(self.loss_fn(out, yt).item())
        acc = float((out.argmax(1) == yt).float().mean().item())
        return loss, acc

    @torch.no_grad()
    def predict(self, x, batch_size: int = 32):
        self.model.eval()
        xt = torch.as_tensor(np.asarray(x, dtype=np.float32))
        outs = [self.model(xt[i:i + batch_size].to(self.exe_device)).cpu() for i in range(0, len(xt), batch_size)]
        return torch.cat(outs).numpy() if outs else np.zeros((0,), np.float32)


class MOON(FedAvgW):
    """One party's worker for the ``moon`` strategy (model-contrastive FL,
    sfl/ml/nn/fl/backend/torch/strategy/moon.py:27-139): local loss = task
    loss + mu * CE(cos(z, z_global) / T against cos(z, z_prev) / T) with the
    model's projection ``z`` (``model(x, return_all=True)`` -> (h, z, y)),
    the aggregated global model and the last ``model_buffer_size`` local
    models.  The aggregation itself is fed_avg_w's: ``average(weights,
    weights=num_samples)`` -- the secure aggregator's caller is unchanged."""

    def __init__(self, builder: TorchModel, device: PYU, random_seed: Optional[int] = None,
                 train_device: Optional[torch.device] = None, model_buffer_size: int = 1, **kwargs):
        super().__init__(builder, device, random_seed, train_device)
        self.model_buffer_size = int(model_buffer_size)
        self.prev_model_list: List[torch.nn.Module] = []
        self.global_model = copy.deepcopy(self.model)

    def train_step(self, weights, cur_steps: int, train_steps: int, refresh_data: bool = False,
                   dp_strategy=None, **kwargs):
        self.model.train()
        if refresh_data:
            self._reset_data_iter()
        if weights is not None:  # moon.py:64-72: global model <- aggregated weights, frozen
            self.set_weights(weights, model=self.global_model)
            self.global_model.eval()
            for prm in self.global_model.parameters():
                prm.requires_grad = False
            self.set_weights(weights)
        num_sample = 0
        loss = None
        for _ in range(train_steps):  # moon.py:76-97
            x, y = self.next_batch()
            num_sample += x.shape[0]
            self.optimizer.zero_grad()
            _, pro1, y_pred = self.model(x, return_all=True)
            loss = self.loss_fn(y_pred, y)
            _, pro2, _ = self.global_model(x, return_all=True)
            logits = self.model.cosine_similarity_fn(pro1, pro2).reshape(-1, 1)
            for pre in self.prev_model_list:
                _, pro3, _ = pre(x, return_all=True)
                nega = self.model.cosine_similarity_fn(pro1, pro3)
                logits = torch.cat((logits, nega.reshape(-1, 1)), dim=1)
            logits = logits / self.model.temperature
            labels = torch.zeros(x.size(0), dtype=torch.long, device=x.device)
            loss = loss + self.model.mu * self.loss_fn(logits, labels)
            loss.backward()
            self.optimizer.step()
        self.last_loss = float(loss.item()) if loss is not None else float("nan")
        model_weights = self.get_weights(return_numpy=True)
        if dp_strategy is not None and dp_strategy.model_gdp is not None:
            model_weights = dp_strategy.model_gdp(model_weights)
        # moon.py:115-130: keep the last model_buffer_size local models, frozen
        if len(self.prev_model_list) >= self.model_buffer_size:
            self.prev_model_list.pop(0)
        hist = copy.deepcopy(self.model)
        hist.eval()
        for prm in hist.parameters():
            prm.requires_grad = False
        self.prev_model_list.append(hist)
        return model_weights, num_sample


class FedAvgU(FedAvgW):
    """``fed_avg_u`` worker (sfl/ml/nn/fl/backend/torch/strategy/fed_avg_u.py:
    30-96): clients upload their model UPDATES (new - old weights) and apply
    the aggregated update.  The aggregator sees small signed deltas."""

    def train_step(self, updates, cur_steps: int, train_steps: int, refresh_data: bool = False,
                   dp_strategy=None, **kwargs):
        self.model.train()
        if refresh_data:
            self._reset_data_iter()
        if updates is not None:  # fed_avg_u.py:55-57
            self.set_weights([np.add(w, u) for w, u in zip(self.get_weights(), updates)])
        old = self.get_weights()
        num_sample = 0
        loss = None
        for _ in range(train_steps):
            x, y = self.next_batch()
            num_sample += x.shape[0]
            self.optimizer.zero_grad()
            loss = self.loss_fn(self.model(x), y)
            loss.backward()
            self.optimizer.step()
        self.last_loss = float(loss.item()) if loss is not None else float("nan")
        client_updates = [np.subtract(n, o) for n, o in zip(self.get_weights(), old)]  # :77-80
        if dp_strategy is not None and dp_strategy.model_gdp is not None:
            client_updates = dp_strategy.model_gdp(client_updates)
        return client_updates, num_sample

    def apply_weights(self, updates, **kwargs):
        if updates is not None:
            self.set_weights([np.add(w, u) for w, u in zip(self.get_weights(), updates)])


class FedAvgG(FedAvgW):
    """``fed_avg_g`` worker (sfl/ml/nn/fl/backend/torch/strategy/fed_avg_g.py:
    28-112): clients upload the gradients of the round and step their
    optimizer with the aggregated gradients.  As in the reference,
    ``local_gradients_sum += local_gradients`` (:91) CONCATENATES the
    per-step gradient lists, so with ``aggregate_freq = k`` the payload the
    aggregator sees is k x the parameter list (k x the mask-stream draws per
    round), and ``set_gradients`` zips it with the parameters
    (mixins.py:99-111), i.e. steps with the first local step's aggregated
    gradients.  One deviation, about the reference's plumbing rather than
    the aggregation: the aggregate (float64 out of the secure decode) is cast
    to each parameter's dtype before it becomes ``p.grad`` (the reference
    assigns it as is, which torch rejects for float32 parameters)."""

    def _set_gradients(self, gradients):
        for g, prm in zip(gradients, self.model.parameters()):
            if g is not None:
                prm.grad = torch.from_numpy(np.array(g, copy=True)).to(device=prm.device, dtype=prm.dtype)

    def train_step(self, gradients, cur_steps: int, train_steps: int, refresh_data: bool = False,
                   dp_strategy=None, **kwargs):
        self.model.train()
        if refresh_data:
            self._reset_data_iter()
        if gradients is not None:  # fed_avg_g.py:67-71
            self._set_gradients(gradients)
            self.optimizer.step()
        num_sample = 0
        loss = None
        grad_sum = None
        for _ in range(train_steps):
            self.optimizer.zero_grad()
            x, y = self.next_batch()
            num_sample += x.shape[0]
            loss = self.loss_fn(self.model(x), y)
            loss.backward()
            grads = [None if prm.grad is None else _host_array(prm.grad)
                     for prm in self.model.parameters()]  # mixins.py:91-97
            grad_sum = grads if grad_sum is None else grad_sum + grads  # list += list: concatenation (:91)
        self.last_loss = float(loss.item()) if loss is not None else float("nan")
        if dp_strategy is not None and dp_strategy.model_gdp is not None:
            grad_sum = dp_strategy.model_gdp(grad_sum)
        return grad_sum, num_sample

    def apply_weights(self, gradients, **kwargs):
        if gradients is not None:  # fed_avg_g.py:103-112
            self._set_gradients(gradients)
            self.optimizer.step()


_STRATEGIES = {("fed_avg_w", "torch"): FedAvgW, ("fed_avg_u", "torch"): FedAvgU, ("fed_avg_g", "torch"): FedAvgG,
               ("moon", "torch"): MOON}


class FLModel:
    """Horizontal FL over ``device_list`` with ``aggregator`` (any object with
    the ``Aggregator`` surface: ``average(data, axis, weights)``)."""

    def __init__(self, server: Optional[PYU] = None, device_list: List[PYU] = (), model: TorchModel = None,
                 aggregator=None, strategy: str = "fed_avg_w", backend: str = "torch",
                 random_seed: Optional[int] = None, train_device=None, dp_strategy=None, **kwargs):
        if (strategy, backend) not in _STRATEGIES:
            raise NotImplementedError(f"strategy {strategy!r} / backend {backend!r}")
        if aggregator is None:
            raise ValueError("this build aggregates through an Aggregator (server_agg_method is out of scope)")
        self.server = server
        self.device_list = list(device_list)
        self._aggregator = aggregator
        self.strategy = strategy
        self.dp_strategy = dp_strategy
        self._workers: Dict[PYU, FedAvgW] = {
            d: _STRATEGIES[(strategy, backend)](model, d, random_seed, train_device, **kwargs)
            for d in self.device_list}

    def initialize_weights(self):
        """Average the clients' initial weights through the aggregator and
        install the result on every worker (reference fl_model.py:126-138):
        one secure aggregation before the first round, which also advances
        every pair's mask streams by the model's parameter count."""
        ws = [PYUObject(d, w.get_weights()) for d, w in self._workers.items()]
        init = self._aggregator.average(ws, axis=0)
        for d, w in self._workers.items():
            w.set_weights(reveal(init.to(d)))
        return init

    def fit(self, x: Dict[PYU, np.ndarray], y: Dict[PYU, np.ndarray], batch_size: int = 32, epochs: int = 1,
            aggregate_freq: int = 1, validation_data=None, round_hook: Callable | None = None) -> dict:
        """``round_hook(round_index, aggregated_params)`` is called after every
        aggregation, with index -1 for the initial-weights average (the test
        oracle checks rounds with it)."""
        for d, w in self._workers.items():
            w.set_data(x[d], y[d], batch_size)
        steps = max(w.steps_per_epoch() for w in self._workers.values())
        history = {"train_loss": [], "val_loss": [], "val_accuracy": [], "aggregation_s": [], "round_s": [],
                   "init_s": 0.0, "eval_s": 0.0}
        # reference fit (fl_model.py:473): the initial weights are averaged
        # through the aggregator before the first epoch
        t_init = time.perf_counter()
        init = self.initialize_weights()
        history["init_s"] = time.perf_counter() - t_init
        if round_hook is not None:
            round_hook(-1, reveal(init))
        rnd = 0
        for epoch in range(epochs):
            model_params_list = None
            for step in range(0, steps, aggregate_freq):
                t_round = time.perf_counter()
                params, nums = [], []
                for idx, (d, w) in enumerate(self._workers.items()):
                    cp = reveal(model_params_list[idx]) if model_params_list is not None else None
                    n_steps = aggregate_freq if step + aggregate_freq < steps else steps - step
                    p, n = w.train_step(cp, epoch * steps + step, n_steps, refresh_data=(step == 0),
                                        dp_strategy=self.dp_strategy)
                    params.append(PYUObject(d, p))
                    nums.append(n)
                t_agg = time.perf_counter()
                model_params = self._aggregator.average(params, axis=0, weights=nums)
                agg_data = reveal(model_params)
                if isinstance(agg_data, list) and agg_data and isinstance(agg_data[0], torch.Tensor):
                    torch.cuda.synchronize()
                history["aggregation_s"].append(time.perf_counter() - t_agg)
                model_params_list = [model_params.to(d) for d in self.device_list]
                history["round_s"].append(time.perf_counter() - t_round)
                if round_hook is not None:
                    round_hook(rnd, agg_data)
                rnd += 1
            for idx, (d, w) in enumerate(self._workers.items()):
                w.apply_weights(reveal(model_params_list[idx]))
            history["train_loss"].append(float(np.mean([w.last_loss for w in self._workers.values()])))
            if validation_data is not None:
                t_eval = time.perf_counter()
                vl, va = self.evaluate(*validation_data)
                history["eval_s"] += time.perf_counter() - t_eval
                history["val_loss"].append(vl)
                history["val_accuracy"].append(va)
        return history

    def evaluate(self, x, y):
        """Global model metrics: after ``fit`` every party holds the same
        aggregated weights, so the first worker evaluates."""
        w = next(iter(self._workers.values()))
        return w.evaluate(x, y)

    def predict(self, x: Dict[PYU, np.ndarray], batch_size: int = 32) -> Dict[PYU, PYUObject]:
        """Every party's predictions on its own data (reference fl_model.py
        ``predict``: a dict device -> PYUObject)."""
        return {d: PYUObject(d, self._workers[d].predict(x[d], batch_size)) for d in self.device_list}

    def get_weights(self, device: Optional[PYU] = None):
        d = device or self.device_list[0]
        return self._workers[d].get_weights()
