"""sfl_amd — MI355X-native secure-aggregation gradient path (drop-in for the
SecureAggregator plugin surface of secretflow/sfl).

Layout:
  csrc/                      HIP kernels (gfx950) + C-ABI (include/sfl_sa.h)
  _lib.py                    ctypes binding of libsfl_sa.so (no fallback)
  kernels.py                 tensor-level wrappers of the C-ABI
  device.py                  PYU / PYUObject / reveal (party runtime slice)
  security/aggregation/      Aggregator ABC, SecureAggregator, Masker
  parallel_sum.py            one-process-per-GPU masked-sum reduce over RCCL
"""

__version__ = "0.1.0"
