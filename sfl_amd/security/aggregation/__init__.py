"""Aggregator plugin surface (mirrors sfl/security/aggregation + the
un-vendored secretflow.security.aggregation)."""
from .aggregator import Aggregator  # noqa: F401
from .masker import Masker  # noqa: F401
from .secure_aggregator import SecureAggregator  # noqa: F401
