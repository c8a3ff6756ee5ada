"""Minimal party/device runtime mirroring the slice of ``secretflow.device``
the aggregator plugin surface touches: ``PYU(party)``, ``PYUObject.to(dev)``,
``dev(fn)(*args)`` and ``reveal``.

In the reference these come from the un-vendored ``secretflow`` package and
run each party in its own Ray/RayFed process.  Here a
party is a name bound to one GPU of this node; objects are plain host or
device values tagged with their owner.  Cross-party movement is explicit
(``.to``), just as in the reference, so aggregator code reads the same.
"""

from __future__ import annotations

from typing import Any, Callable

import numpy as np


class PYU:
    """A party's compute device: party name + GPU index (``None`` = CPU only)."""

    def __init__(self, party: str, gpu: int | None = 0):
        self.party = str(party)
        self.gpu = gpu

    @property
    def torch_device(self):
        import torch

        return torch.device("cuda", self.gpu) if self.gpu is not None else torch.device("cpu")

    def __call__(self, fn: Callable, num_returns: int | None = None, **_kw):
        def run(*args, **kwargs):
            a = [_local(x, self) for x in args]
            k = {key: _local(v, self) for key, v in kwargs.items()}
            out = fn(*a, **k)
            if num_returns is not None and num_returns > 1:
                return [PYUObject(self, o) for o in out]
            return PYUObject(self, out)

        return run

    def __eq__(self, other):
        return isinstance(other, PYU) and other.party == self.party

    def __hash__(self):
        return hash(("PYU", self.party))

    def __repr__(self):
        return f"PYU({self.party!r}, gpu={self.gpu})"


class PYUObject:
    """A value owned by one party."""

    def __init__(self, device: PYU, data: Any):
        self.device = device
        self.data = data

    def to(self, device: PYU) -> "PYUObject":
        return PYUObject(device, _move(self.data, device))

    def __repr__(self):
        return f"PYUObject(device={self.device!r})"


DeviceObject = PYUObject


def _local(x, dev: PYU):
    """Resolve device objects in ``x`` -- nested in lists, tuples and dicts
    too, as secretflow flattens a call's arguments -- to their values."""
    if isinstance(x, PYUObject):
        if x.device != dev:
            raise ValueError(f"{x.device} object used on {dev}; move it with .to() first")
        return x.data
    if isinstance(x, (list, tuple)):
        return _rebuild(x, [_local(v, dev) for v in x])
    if isinstance(x, dict):
        return {k: _local(v, dev) for k, v in x.items()}
    return x


def _rebuild(x, items: list):
    """``x`` (a list or tuple, possibly a subclass) with its elements replaced
    by ``items``: ``x`` itself when nothing changed (so any subclass passes
    through as before), a namedtuple from positional fields, otherwise
    ``type(x)(items)``."""
    if all(a is b for a, b in zip(x, items)):
        return x
    if hasattr(x, "_fields"):  # namedtuple: fields are positional arguments
        return type(x)(*items)
    return type(x)(items)


def _move(data, dev: PYU):
    try:
        import torch
    except ImportError:  # pragma: no cover
        torch = None
    if isinstance(data, (list, tuple)):
        return _rebuild(data, [_move(d, dev) for d in data])
    if isinstance(data, dict):
        return {k: _move(v, dev) for k, v in data.items()}
    if torch is not None and isinstance(data, torch.Tensor):
        if data.device.type == "cpu" and dev.torch_device.type == "cuda" and not data.requires_grad:
            from . import hostpipe as H  # a pinned copy, never a pageable DMA (hostpipe.d2h)

            if H.host_dtype(data) is not None:
                return H.h2d(data, dev.torch_device)
        return data.to(dev.torch_device)
    if isinstance(data, np.ndarray):
        return data.copy()
    return data


def reveal(obj):
    """Bring a party-owned value to the driver (host)."""
    if isinstance(obj, (list, tuple)):
        return type(obj)(reveal(o) for o in obj)
    if isinstance(obj, PYUObject):
        return obj.data
    return obj
