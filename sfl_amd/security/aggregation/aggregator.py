"""The aggregator plugin interface.

Mirrors ``secretflow.security.aggregation.Aggregator`` (un-vendored), whose
shape is pinned in-tree by its implementations
``sfl/security/aggregation/sparse_plain_aggregator.py:75,98``,
``sfl/security/aggregation/experiment/ppb_aggregator.py:294,342`` and the ABC
mirror ``sfl_lite/sfl_lite/security/aggregation/aggregator.py:21-32``.
"""

from __future__ import annotations

from abc import ABC, abstractmethod
from typing import List

from ...device import DeviceObject


class Aggregator(ABC):
    """The abstract aggregator."""

    @abstractmethod
    def sum(self, data: List[DeviceObject], axis=None) -> DeviceObject:
        """Sum of array elements over a given axis (axis=0: over parties)."""

    @abstractmethod
    def average(self, data: List[DeviceObject], axis=None, weights=None) -> DeviceObject:
        """Weighted average over a given axis (axis=0: over parties)."""
