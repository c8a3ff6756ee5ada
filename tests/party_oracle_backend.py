"""CPU stand-in for the two device steps of ``sfl_amd.security.aggregation.party``
-- TEST INFRASTRUCTURE ONLY (it calls the numpy oracle).

The CPU suite has no GPU, so ``install()`` (run first inside each spawned
party process of ``tests/fake_secretflow.py``) swaps ``party._mask_vector``
and ``party._sum_decode_vectors`` for the oracle's arithmetic.  Everything
else -- who creates which masker, what is revealed, what moves where, stream
positions, dtype promotion, digests -- is the product code under test.  The
``-m gpu`` tests run the same protocol with the HIP steps."""
from __future__ import annotations

import numpy as np


def install():
    from sfl_amd.security.aggregation import party as P

    P._mask_vector = _mask_vector
    P._sum_decode_vectors = _sum_decode_vectors


def _mask_vector(masker, xs, xt, ct, wscalar, wvec, gpu):
    from oracle import secagg as o
    from sfl_amd import _lib as L

    x = np.concatenate([np.asarray(a, dtype=xt).reshape(-1) for a in xs]).astype(ct)
    with np.errstate(over="ignore", invalid="ignore"):
        if wvec is not None:
            d = x * np.asarray(wvec, dtype=ct)
        else:
            d = x * (ct.type(wscalar))
        d = d * ct.type(1 << masker.fxp_bits)
    q = o.quantize(d, None, 0)
    out = q.copy()
    extra = {}
    for peer in masker.peers:
        g0 = masker.generator(peer)
        g = o.generator_from_state(*g0.pair())
        m = g.integers(o.INT64_MIN, o.INT64_MAX, size=out.size).astype(np.uint64)
        if masker.sign(peer) > 0:
            out += m
        else:
            out -= m
        st = g.bit_generator.state["state"]["state"]
        k = 0
        while L.pcg64_advance(g0, out.size + k).pair()[0] != st:
            k += 1
            assert k < 64, "stream position lost"
        if k:
            extra[peer] = k
    return out, extra, None  # no device digest: mask_payload XORs the host vector


def _sum_decode_vectors(u64s, digests, fxp_bits, divisor, divisor_vec, gpu, as_torch):
    from oracle import secagg as o
    from sfl_amd.security.aggregation.party import DigestMismatch

    for i, (u, d) in enumerate(zip(u64s, digests)):
        if o.digest(u) != int(d):
            raise DigestMismatch(f"masked vector {i}")
    s = o.server_sum(u64s)
    div = divisor if divisor_vec is None else np.sum(np.stack(divisor_vec), axis=0)
    return o.decode(s, fxp_bits, div)
