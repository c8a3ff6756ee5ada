"""Reference-side import path: the HIP ``SecureAggregator`` for code written
against ``secretflow`` (missing 5).

Callers import ``from secretflow.security import SecureAggregator``
(``tests/ml/nn/fl/strategy/test_moon_torch.py:17``,
``sfl/security/aggregation/stateful_fedgen_aggregator.py:20``) and hand it
secretflow devices and device objects: ``PYU`` objects carrying ``.party``,
``PYUObject`` objects carrying ``.device`` whose value the driver fetches
with ``sf.reveal`` (simulation mode), and results that come back as objects
on the server device.  This module accepts exactly those shapes, duck-typed
(secretflow itself is not installed here):

* ``SecureAggregator(device, participants, fxp_bits=18)`` -- the reference
  constructor; devices map to ``sfl_amd.device.PYU`` by party name, each on
  the GPU ``gpu_of(party)`` picks (default: every party on GPU 0, the
  single-node simulation);
* ``sum(data, axis)`` / ``average(data, axis, weights)`` -- data are
  secretflow-shaped objects (or already ``sfl_amd`` ones); their values
  are fetched with ``reveal`` (default: ``secretflow.reveal`` when
  importable), weights may be plain numbers / arrays or device objects on
  the matching party (``stateful_fedgen_aggregator.py:74-78`` puts them on
  the client's device);
* the result is wrapped back onto the server device with ``wrap(device,
  value)`` (default: ``device(lambda v: v)(value)``, which is how a
  secretflow ``PYU`` creates a ``PYUObject`` it owns).

``install(module)`` rebinds ``module.SecureAggregator`` (e.g.
``secretflow.security.aggregation`` or ``secretflow.security``), so existing
call sites pick up the HIP path unchanged; INTEGRATION.md §5 shows it.
"""

from __future__ import annotations

from typing import Callable, List, Optional

from ..device import PYU, PYUObject, reveal as _reveal_local
from ..security.aggregation import SecureAggregator as _HipSecureAggregator


def _default_reveal():
    try:  # pragma: no cover - secretflow is not installed in this image
        import secretflow as sf

        return sf.reveal
    except ImportError:
        return None


def _default_wrap(device, value):
    return device(lambda v: v)(value)


class SecureAggregator:
    """secretflow-shaped front of the HIP secure aggregator."""

    def __init__(self, device, participants: List, fxp_bits: int = 18, *,
                 reveal: Optional[Callable] = None, wrap: Optional[Callable] = None,
                 gpu_of: Optional[Callable[[str], int]] = None, **kwargs):
        self._sf_device = device
        self._sf_participants = list(participants)
        self._reveal = reveal or _default_reveal()
        self._wrap = wrap or _default_wrap
        gpu_of = gpu_of or (lambda party: 0)
        self._pyu = {}
        for d in [device] + self._sf_participants:
            party = _party(d)
            if party not in self._pyu:
                self._pyu[party] = PYU(party, gpu_of(party))
        self._inner = _HipSecureAggregator(self._pyu[_party(device)],
                                           [self._pyu[_party(p)] for p in self._sf_participants],
                                           fxp_bits, **kwargs)

    @property
    def device(self):
        return self._sf_device

    @property
    def participants(self):
        return list(self._sf_participants)

    @property
    def inner(self) -> _HipSecureAggregator:
        """The sfl_amd aggregator doing the work (digests, wire images)."""
        return self._inner

    def sum(self, data: List, axis=None):
        out = self._inner.sum(self._objects(data), axis=axis)
        return self._wrap(self._sf_device, _reveal_local(out))

    def average(self, data: List, axis=None, weights=None):
        if weights is not None and not _is_device_object(weights):
            assert len(weights) == len(data), (
                f"Length of the weights does not match the data: {len(weights)} vs {len(data)}.")
            for i, w in enumerate(weights):
                # a device-object weight must live on its data's party
                # (stateful_fedgen_aggregator.py:74-78), checked before it is revealed
                if _is_device_object(w) and _is_device_object(data[i]):
                    assert _party(w.device) == _party(data[i].device), (
                        "Device of weight does not match the corresponding data device.")
            weights = [self._value(w) if _is_device_object(w) else w for w in weights]
        out = self._inner.average(self._objects(data), axis=axis, weights=weights)
        return self._wrap(self._sf_device, _reveal_local(out))

    # ------------------------------------------------------------ internals
    def _value(self, obj):
        if isinstance(obj, PYUObject):
            return obj.data
        if self._reveal is None:
            raise RuntimeError("secretflow device objects need a reveal function (pass reveal=sf.reveal)")
        return self._reveal(obj)

    def _objects(self, data):
        assert data, "Data to aggregate should not be None or empty!"
        out = []
        for d in data:
            if isinstance(d, PYUObject):
                out.append(d)
                continue
            if not _is_device_object(d):
                raise TypeError(f"expect a device object (with .device), got {type(d)}")
            party = _party(d.device)
            if party not in self._pyu:
                raise AssertionError(f"{d.device} is not a participant")
            out.append(PYUObject(self._pyu[party], self._value(d)))
        return out


def _party(device) -> str:
    party = getattr(device, "party", None)
    if party is None:
        raise TypeError(f"expect a secretflow PYU-like device with .party, got {type(device)}")
    return str(party)


def _is_device_object(x) -> bool:
    return hasattr(x, "device") and hasattr(getattr(x, "device"), "party")


def install(module) -> None:
    """Rebind ``module.SecureAggregator`` to the HIP aggregator, e.g.::

        import secretflow.security.aggregation as agg
        from sfl_amd.compat import secretflow as hip
        hip.install(agg)            # every later SecureAggregator(...) runs on MI355X
    """
    module.SecureAggregator = SecureAggregator
