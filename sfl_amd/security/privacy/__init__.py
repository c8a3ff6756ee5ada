"""Differential-privacy pre-step of the FL secure-aggregation path
(mirrors sfl/security/privacy)."""
from .mechanism import DPStrategyFL, GaussianModelDP  # noqa: F401
