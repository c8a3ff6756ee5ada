"""Host-side check of the masking kernel's accumulator algebra (no GPU).

k_clients (sfl_amd/csrc/sa_clients_impl.h) keeps the upper half of the L
co-located clients NEGATED in their accumulators (``negated<L>``) so that
an internal pair (u, v) -- +t to u, -t to v -- becomes two one-instruction
adds when u is in the lower and v in the upper half (``Sched::role``).  A
negated client's cross streams draw ~t (sign mask inverted) and its
accumulator starts at X - bias; the finish forms q - st.

This restates those rules over Python integers mod 2^64 for every fused
shape the library instantiates and checks each client's masked value
against the direct formula  bias_c + q_c + sum(+t for pairs where c is u)
- sum(t for pairs where c is v) + sum(cross t), i.e. what the kernel
computed before the change (and what the oracle's per-client masks sum
to; the GPU parity tests pin the kernel itself bit for bit)."""
import random

import pytest

M = (1 << 64) - 1
SHAPES = [(L, 0) for L in range(1, 9)] + [(4, 4), (2, 6), (2, 2)] + [(1, x) for x in range(0, 17)]


def negated(L, c):
    return L >= 2 and c >= L // 2


def pairs(L):
    return [(u, v) for u in range(L) for v in range(u + 1, L)]


def role(L, X, q):
    """Mirror of Sched<L, X>::role: (add target, partner, partner adds, flip)."""
    PI = len(pairs(L))
    if q >= PI:
        c = (q - PI) // (X if X > 0 else 1)
        return c, -1, False, negated(L, c)
    u, v = pairs(L)[q]
    if not negated(L, v):
        return u, v, False, False
    if not negated(L, u):
        return u, v, True, False
    return v, u, False, False


@pytest.mark.parametrize("L,X", sorted(set(SHAPES)))
def test_negated_storage_equals_direct_formula(L, X):
    rng = random.Random(1000 * L + X)
    PI = len(pairs(L))
    P = PI + L * X
    for _ in range(20):
        raw = [rng.getrandbits(64) for _ in range(P)]
        smask = [rng.choice([0, M]) for _ in range(P)]
        bias = [rng.getrandbits(64) for _ in range(L)]
        q = [rng.getrandbits(64) for _ in range(L)]
        # direct (reference orientation): t = raw ^ smask; u += t, v -= t, cross c += t
        direct = [(bias[c] + q[c]) & M for c in range(L)]
        for p, (u, v) in enumerate(pairs(L)):
            t = raw[p] ^ smask[p]
            direct[u] = (direct[u] + t) & M
            direct[v] = (direct[v] - t) & M
        for c in range(L):
            for j in range(X):
                t = raw[PI + c * X + j] ^ smask[PI + c * X + j]
                direct[c] = (direct[c] + t) & M
        # kernel: storage init, one add per target (or add + subtract), finish
        st = [((X - bias[c]) if negated(L, c) else bias[c]) & M for c in range(L)]
        for qi in range(P):
            a, b, b_add, flip = role(L, X, qi)
            t = raw[qi] ^ smask[qi] ^ (M if flip else 0)
            st[a] = (st[a] + t) & M
            if b >= 0:
                st[b] = (st[b] + t) & M if b_add else (st[b] - t) & M
        fin = [((q[c] - st[c]) if negated(L, c) else (st[c] + q[c])) & M for c in range(L)]
        assert fin == direct


def test_half_of_the_pairs_add_twice():
    """8 clients: 16 of the 28 internal pairs add to both accumulators."""
    assert sum(role(8, 0, q)[2] for q in range(28)) == 16
    assert sum(role(4, 0, q)[2] for q in range(6)) == 4
    assert role(2, 0, 0)[2]
