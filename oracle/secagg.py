"""CPU oracle for the secure-aggregation hot path — TEST INFRASTRUCTURE ONLY.

This module restates, in plain numpy, the element-wise algorithm of
``secretflow.security.aggregation.SecureAggregator`` / ``_Masker`` (the
un-vendored third-party package ``secretflow-lite==1.13.0b0`` pinned at
``/root/reference/pyproject.toml:51`` and ``uv.lock:2008-2009``).  It is the
checker the HIP path is compared against; it is never the thing measured or
shipped.  Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s
``cpu_baseline`` leg (``benchkit/baseline.py``) may import it.  The product path (``sfl_amd``) must never
import this file — ``tests/test_boundary.py`` enforces that.

Where the algorithm is pinned (all paths relative to /root/reference):

* masking equation ``y_u = x_u + sum_{u<v} s_uv - sum_{u>v} s_uv  mod R``:
  ``docs/developer/algorithm/secure_aggregation.ipynb`` cell 15 (json lines
  225-245 of the notebook source); PRG = ``numpy.random.PCG64`` (same cell).
* fixed-point scale is a power of two, ``fxp_bits = 18`` by default:
  ``CHANGELOG.md:1111`` and ``sfl/security/aggregation/stateful_fedgen_aggregator.py:29-32``.
* quantizer = truncation toward zero, decoded dtype float64: the notebook's
  known-answer outputs (cells 17-18) reproduce to <5e-9 only with trunc; see
  ``tests/golden/notebook_kat.json``.
* per-element (multi-dimensional) weights: ``CHANGELOG.md:994`` and
  ``tests/security/aggregation/test_aggregator_base.py:144-160``.
* server sum = ``np.sum(list_of_uint64, axis=0)`` wrapping mod 2^64, the
  pattern of ``sfl/security/aggregation/sparse_plain_aggregator.py:88-94``.

The arithmetic dependency is numpy itself (PCG64, SeedSequence,
``Generator.integers`` with Lemire bounded draws, uint64 wrap-around): this
oracle calls numpy's own generator, so its mask streams are the reference's
mask streams bit for bit for the same seeds.
"""

from __future__ import annotations

import numpy as np

FXP_BITS = 18
INT64_MIN = np.iinfo(np.int64).min
INT64_MAX = np.iinfo(np.int64).max
U64 = (1 << 64) - 1
PCG64_MULT = 0x2360ED051FC65DA44385DF649FCCF645
# Generator.integers(int64.min, int64.max) == raw + MASK_OFFSET (mod 2^64); raw==0 is rejected.
MASK_OFFSET = 0x7FFFFFFFFFFFFFFF
BENCH_SEED_TAG = 0x5ECA66


def pair_seed(u: int, v: int, tag: int = BENCH_SEED_TAG) -> int:
    """Deterministic pairwise seed used by the benches and golden fixtures
    (SURVEY.md §8(d)): ``(tag << 32) | (min << 16) | max``.  The reference
    derives this from a Diffie-Hellman secret (un-vendored); any seed works
    because the masks cancel."""
    a, b = (u, v) if u < v else (v, u)
    return (tag << 32) | (a << 16) | b


def pcg64_state(seed) -> tuple[int, int]:
    """(state, inc) of ``np.random.default_rng(seed)`` — i.e. PCG64 seeded
    through SeedSequence, exactly what the reference's ``_Masker`` builds."""
    st = np.random.default_rng(seed).bit_generator.state["state"]
    return int(st["state"]), int(st["inc"])


def mask_stream(seed, n: int, offset: int = 0) -> np.ndarray:
    """The uint64 mask a ``_Masker`` adds for one peer:
    ``default_rng(seed).integers(int64.min, int64.max, n).astype(uint64)``,
    taken after ``offset`` earlier draws (earlier aggregation rounds)."""
    bg = np.random.PCG64(seed)
    if offset:
        bg.advance(offset)
    g = np.random.Generator(bg)
    return g.integers(INT64_MIN, INT64_MAX, size=n).astype(np.uint64)


def quantize(x: np.ndarray, weight=None, fxp_bits: int = FXP_BITS) -> np.ndarray:
    """``trunc(x * w * 2^fxp)`` as int64, viewed as uint64 (two's complement).

    numpy promotion rules decide the arithmetic type as in the reference's
    pinned numpy 1.23.5: float32 data with a python-int weight stays float32,
    and so does float32 data with a numpy-scalar weight (value-based casting,
    ``legacy_scalar_dtype``); an int64 weight array promotes float32 data to
    float64; int data stays int64.
    Non-finite or out-of-int64-range values map to INT64_MIN, which is what
    ``ndarray.astype(np.int64)`` yields on x86-64 (cvttsd2si "integer
    indefinite"); we spell it out so the oracle is platform independent."""
    x = np.asarray(x)
    with np.errstate(over="ignore", invalid="ignore"):
        if weight is None:
            d = x
        elif (isinstance(weight, (bool, int, float)) and not isinstance(weight, np.generic)) or np.ndim(weight):
            d = x * weight
        else:  # numpy scalar / 0-d weight: numpy 1.23.5's value-based casting
            d = np.multiply(x, weight, dtype=legacy_scalar_dtype(x.dtype, weight))
        d = d * (1 << fxp_bits)
    if np.issubdtype(d.dtype, np.integer):
        return d.astype(np.int64).astype(np.uint64)
    d = np.asarray(d)
    ok = np.abs(d.astype(np.float64)) < 2.0**63  # False for NaN/inf/out of range
    t = np.trunc(np.where(ok, d, 0))
    q = t.astype(np.int64)
    q = np.where(ok, q, np.int64(INT64_MIN))
    return q.astype(np.int64).astype(np.uint64)


def legacy_scalar_dtype(x_dtype, scalar) -> np.dtype:
    """``array * numpy_scalar`` result dtype under numpy 1.23.5, the version
    the reference pins (``uv.lock:1189-1190``): value-based casting -- the
    scalar takes part with the smallest dtype that holds its value
    (``np.min_scalar_type``), so float32 data times ``np.float64(3.0)`` or
    ``np.int64(5)`` stays float32 (numpy 2's NEP 50 would give float64)."""
    return np.result_type(np.dtype(x_dtype), np.min_scalar_type(np.asarray(scalar)))


def mask_client(q: np.ndarray, self_name, peer_seeds: dict, offset: int = 0) -> np.ndarray:
    """Apply pairwise masks to one client's quantized vector:
    ``+= m`` for every peer whose name sorts after ours, ``-= m`` otherwise
    (the ``party > self._party`` rule of the notebook's equation)."""
    out = np.array(q, dtype=np.uint64, copy=True).reshape(-1)
    n = out.size
    for peer, seed in peer_seeds.items():
        if peer == self_name:
            continue
        m = mask_stream(seed, n, offset)
        if peer > self_name:
            out += m
        else:
            out -= m
    return out.reshape(np.shape(q))


def server_sum(masked: list) -> np.ndarray:
    """Server-side ``np.sum(masked, axis=0)`` over uint64, wrapping mod 2^64."""
    return np.sum(np.stack([np.asarray(m, dtype=np.uint64) for m in masked]), axis=0, dtype=np.uint64)


def decode(s: np.ndarray, fxp_bits: int = FXP_BITS, divisor=None) -> np.ndarray:
    """``s.astype(int64) / 2^fxp`` as float64, then ``/ divisor`` (Σw or C)."""
    out = np.asarray(s, dtype=np.uint64).astype(np.int64) / (1 << fxp_bits)
    if divisor is not None:
        out = out / divisor
    return out


def digest(masked: np.ndarray) -> int:
    """XOR of every uint64 element of a masked vector — the size-independent
    per-client checksum the fused HIP kernel reports."""
    a = np.asarray(masked, dtype=np.uint64).reshape(-1)
    if a.size == 0:
        return 0
    return int(np.bitwise_xor.reduce(a))


def checksum(v: np.ndarray) -> int:
    """Sum of uint64 elements mod 2^64 (checksum of a sum vector)."""
    a = np.asarray(v, dtype=np.uint64).reshape(-1)
    return int(np.sum(a, dtype=np.uint64)) if a.size else 0


def seeds_for(names: list, seed_fn=None) -> dict:
    """Pairwise seed table {name: {peer: seed}} for clients ``names``."""
    seed_fn = seed_fn or (lambda i, j: pair_seed(i, j))
    idx = {n: i for i, n in enumerate(names)}
    return {
        a: {b: seed_fn(idx[a], idx[b]) for b in names if b != a} for a in names
    }


def secure_masked(xs: list, names: list, weights=None, fxp_bits: int = FXP_BITS,
                  seeds: dict | None = None, offset: int = 0) -> list:
    """Every client's masked uint64 vector (what crosses the wire)."""
    seeds = seeds or seeds_for(names)
    out = []
    for i, (x, name) in enumerate(zip(xs, names)):
        w = None if weights is None else weights[i]
        q = quantize(x, w, fxp_bits)
        out.append(mask_client(q, name, seeds[name], offset))
    return out


def secure_sum(xs: list, names: list, fxp_bits: int = FXP_BITS, seeds=None, offset: int = 0):
    """Decoded secure sum (float64) and the integer masked sum."""
    masked = secure_masked(xs, names, None, fxp_bits, seeds, offset)
    s = server_sum(masked)
    return decode(s, fxp_bits), s, masked


def secure_average(xs: list, names: list, weights=None, fxp_bits: int = FXP_BITS,
                   seeds=None, offset: int = 0):
    """Decoded secure average: ``Σ q(x_c w_c) / 2^fxp / Σ w_c`` (``/ C``
    without weights); per-element weights divide element-wise."""
    masked = secure_masked(xs, names, weights, fxp_bits, seeds, offset)
    s = server_sum(masked)
    if weights is None:
        div = len(xs)
    else:
        div = np.sum(np.stack([np.asarray(w) for w in weights]), axis=0) if np.ndim(weights[0]) else sum(weights)
    return decode(s, fxp_bits, div), s, masked


# ----- pure-python PCG64 restatement (small cases; pins the HIP stepping) -----

def pcg64_raw_py(state: int, inc: int, n: int) -> list:
    """numpy's ``pcg_setseq_128_xsl_rr_64``: step the 128-bit LCG, then
    XSL-RR the NEW state.  Pure python; only for small n."""
    out = []
    s = state
    for _ in range(n):
        s = (s * PCG64_MULT + inc) & ((1 << 128) - 1)
        hi, lo = s >> 64, s & U64
        r = hi >> 58
        x = hi ^ lo
        out.append(((x >> r) | (x << ((64 - r) & 63))) & U64)
    return out


def pcg64_jump_py(state: int, inc: int, delta: int) -> int:
    """State after ``delta`` steps (== ``PCG64.advance(delta)``), by
    square-and-multiply of the affine map s -> A s + inc."""
    M = (1 << 128) - 1
    acc_mult, acc_plus = 1, 0
    cur_mult, cur_plus = PCG64_MULT, inc
    d = delta & M
    while d:
        if d & 1:
            acc_mult = (acc_mult * cur_mult) & M
            acc_plus = (acc_plus * cur_mult + cur_plus) & M
        cur_plus = ((cur_mult + 1) * cur_plus) & M
        cur_mult = (cur_mult * cur_mult) & M
        d >>= 1
    return (acc_mult * state + acc_plus) & M


# ----- persistent per-party generators (the reference _Masker's view) -----

def generator_from_state(state: int, inc: int) -> np.random.Generator:
    """numpy Generator over PCG64 with an explicit (state, inc)."""
    bg = np.random.PCG64()
    bg.state = {"bit_generator": "PCG64", "state": {"state": int(state), "inc": int(inc)},
                "has_uint32": 0, "uinteger": 0}
    return np.random.Generator(bg)


class OracleMaskers:
    """Every party's persistent ``np.random.Generator`` per peer, advanced by
    ``Generator.integers(int64.min, int64.max, n)`` round after round --
    numpy's own rejection of a raw 0 included, exactly as the un-vendored
    ``_Masker`` keeps one generator per peer across rounds.  ``pair_states``
    maps (a, b) -> seed (int) or (state, inc)."""

    def __init__(self, names: list, pair_states: dict):
        self.names = list(names)
        self.gens = {}
        for a in names:
            for b in names:
                if a == b:
                    continue
                st = pair_states.get((a, b), pair_states.get((b, a)))
                self.gens[(a, b)] = (generator_from_state(*st) if isinstance(st, tuple)
                                     else np.random.Generator(np.random.PCG64(st)))

    def mask(self, q: np.ndarray, me: str) -> np.ndarray:
        out = np.array(q, dtype=np.uint64, copy=True).reshape(-1)
        for peer in sorted(p for p in self.names if p != me):
            m = self.gens[(me, peer)].integers(INT64_MIN, INT64_MAX, size=out.size).astype(np.uint64)
            if peer > me:
                out += m
            else:
                out -= m
        return out

    def round(self, xs: list, weights=None, fxp_bits: int = FXP_BITS):
        """(masked vectors, uint64 sum) of one round; xs in ``names`` order."""
        masked = [self.mask(quantize(x, None if weights is None else weights[i], fxp_bits), nm)
                  for i, (x, nm) in enumerate(zip(xs, self.names))]
        return masked, server_sum(masked)
