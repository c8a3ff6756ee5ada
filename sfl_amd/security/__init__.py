from .aggregation import Aggregator, SecureAggregator  # noqa: F401
