"""GaussianModelDP on the GPU (the DP pre-step of the
secure-aggregation path).

Mirrors ``sfl/security/privacy/mechanism/mechanism_fl.py:26-130``: the
client's list of float32 arrays is clipped to the global L2 norm
(``scale = min(1, clip / ||all||)``, or per layer ``min(1, clip /
sqrt(||layer|| * ||all||))`` with ``is_clip_each_layer``) and
``N(0, sigma^2) / num_updates`` is added, ``sigma = noise_multiplier *
l2_norm_clip * l2_norm_clip`` exactly as the reference writes it.

Device work: ``sa_sumsq_f32`` (each layer's norm as the reference forms it:
np.linalg.norm's float32 norm, squared and summed over the layers in
float64 as numpy 1.23.5 does for these scalars), then
``sa_dp_perturb_f32`` (this class's ``__call__``: the perturbed arrays are
materialised, as the reference returns them).  ``sa_mask_dp`` runs the
same clip + noise inside the masking kernel, bit-identical; the loopback
client uses it (2–3 % faster than perturb-then-mask on MI355X).

The noise is Philox4x32-10 + Box-Muller keyed by a 64-bit key and the
element index (reproducible, parallel), not numpy's unseeded global
``np.random.normal`` stream; the privacy accounting (RDP) is unchanged by
that and is out of scope here.
"""

from __future__ import annotations

import secrets
from typing import List, Optional

import numpy as np
import torch

from ... import _lib as L
from ... import hostpipe as H
from ... import kernels as K


class GaussianModelDP:
    def __init__(self, noise_multiplier: float, num_clients: int, num_updates: Optional[int] = None,
                 l2_norm_clip: float = 1.0, delta: Optional[float] = None, is_secure_generator: bool = False,
                 is_clip_each_layer: bool = False, *, device=None, seed: Optional[int] = None) -> None:
        if is_secure_generator:
            raise NotImplementedError("is_secure_generator: this build draws noise from Philox4x32-10 only")
        self.noise_multiplier = noise_multiplier
        self.l2_norm_clip = l2_norm_clip
        self.num_clients = num_clients
        self.num_updates = num_clients if num_updates is None else num_updates
        self.delta = delta if delta is not None else min(1 / num_clients**2, 1e-5)
        self.is_secure_generator = is_secure_generator
        self.is_clip_each_layer = is_clip_each_layer
        self.device = torch.device(device) if device is not None else torch.device("cuda", 0)
        self.key = secrets.randbits(64) if seed is None else int(seed) & ((1 << 64) - 1)
        self.counter = 0  # noise index of the next element (advances by whole Philox blocks)

    @property
    def noise_std(self) -> float:
        return self.noise_multiplier * self.l2_norm_clip * self.l2_norm_clip

    def _flat(self, a) -> torch.Tensor:
        if isinstance(a, torch.Tensor):
            t = a.detach().to(device=self.device, dtype=torch.float32).reshape(-1).contiguous()
        else:
            t = torch.from_numpy(np.ascontiguousarray(np.asarray(a, dtype=np.float32)).reshape(-1)).to(self.device)
        return t.clone() if t.data_ptr() % 16 else t

    def sumsq(self, xs: List[torch.Tensor]) -> torch.Tensor:
        """``sum([np.linalg.norm(x) ** 2 for x in xs])`` on the device
        (mechanism_fl.py:133): float32 layer norms, float64 squares and sum."""
        out = torch.zeros(1, dtype=torch.float64, device=self.device)
        part = torch.empty(L.SA_DP_PARTIALS, dtype=torch.float64, device=self.device)
        for x in xs:
            if x.numel():
                K.sumsq_f32(x, out, part, accumulate=True)
        return out

    def params(self, sumsq: torch.Tensor, n: int, sumsq_layer: torch.Tensor | None = None) -> L.DP:
        """sa_dp for the next n elements (advances the noise counter)."""
        d = K.make_dp(sumsq, l2_norm_clip=self.l2_norm_clip, noise_std=self.noise_std,
                      num_updates=self.num_updates, key=self.key, counter0=self.counter, sumsq_layer=sumsq_layer)
        self.counter += -(-n // 4) * 4
        return d

    def __call__(self, inputs: List):
        """Clip + noise every array of ``inputs``; numpy in -> numpy out,
        torch in -> torch (float32, on ``device``) out."""
        assert inputs, "the inputs of GaussianModelDP should not be empty!"
        as_torch = isinstance(inputs[0], torch.Tensor)
        shapes = [tuple(a.shape) for a in inputs]
        xs = [self._flat(a) for a in inputs]
        total = self.sumsq(xs)
        part = torch.empty(L.SA_DP_PARTIALS, dtype=torch.float64, device=self.device)
        out = []
        for x, shape in zip(xs, shapes):
            layer = None
            if self.is_clip_each_layer:
                layer = torch.zeros(1, dtype=torch.float64, device=self.device)
                if x.numel():
                    K.sumsq_f32(x, layer, part)
            y = torch.empty_like(x)
            dp = self.params(total, x.numel(), layer)
            if x.numel():
                K.dp_perturb(x, y, dp)
            y = y.reshape(shape)
            out.append(y if as_torch else H.d2h(y, pooled=False))
        return out

    def global_norm(self, inputs) -> float:
        """``np.sqrt(sum(norm ** 2))`` in float64, as the reference's
        ``global_norm`` returns it under numpy 1.23.5 (mechanism_fl.py:132-135)."""
        xs = [self._flat(a) for a in inputs]
        return float(np.sqrt(np.float64(self.sumsq(xs).item())))


class DPStrategyFL:
    """``sfl/security/privacy/strategy_fl.py:18-32`` (accounting out of scope)."""

    def __init__(self, model_gdp: GaussianModelDP = None, accountant_type="rdp"):
        self.model_gdp = model_gdp
        if accountant_type == "rdp":
            self.accountant_type = accountant_type
