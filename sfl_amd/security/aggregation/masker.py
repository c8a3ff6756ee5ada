"""Per-party masking state: pairwise key agreement and PCG64 mask streams.

Replaces the setup half of the un-vendored ``secretflow`` ``_Masker`` actor
(SURVEY.md §3A): each party holds a Diffie-Hellman key pair; every pair of
parties derives a shared secret, hashes it to a 128-bit seed, and builds
``np.random.default_rng(seed)`` — here the equivalent numpy-exact PCG64
state computed by the C-ABI (``sa_pcg64_from_seed``).  The generator position
(how many draws earlier rounds consumed) is tracked per (party, peer), exactly
like the reference's persistent ``Generator`` objects.

The reference's DH group and secret->seed derivation are not in the snapshot
(un-vendored); any derivation works because masks cancel, and tests and
benches may pass explicit seeds instead.
"""

from __future__ import annotations

import hashlib
import secrets

from ... import _lib as L

# RFC 3526 group 14 (2048-bit MODP), generator 2
_P = int(
    "FFFFFFFFFFFFFFFFC90FDAA22168C234C4C6628B80DC1CD129024E088A67CC74020BBEA63B139B22514A08798E3404DD"
    "EF9519B3CD3A431B302B0A6DF25F14374FE1356D6D51C245E485B576625E7EC6F44C42E9A637ED6B0BFF5CB6F406B7ED"
    "EE386BFB5A899FA5AE9F24117C4B1FE649286651ECE45B3DC2007CB8A163BF0598DA48361C55D39A69163FA8FD24CF5F"
    "83655D23DCA3AD961C62F356208552BB9ED529077096966D670C354E4ABC9804F1746C08CA18217C32905E462E36CE3B"
    "E39E772C180E86039B2783A2EC07A28FB5C55DF06F4C52C9DE2BCBF6955817183995497CEA956AE515D2261898FA0510"
    "15728E5A8AACAA68FFFFFFFFFFFFFFFF", 16)
_G = 2


class DiffieHellman:
    def __init__(self):
        self._priv = secrets.randbits(256) | 1
        self.public_key = pow(_G, self._priv, _P)

    def shared_seed(self, peer_public: int) -> int:
        if not 1 < peer_public < _P - 1:
            raise ValueError("invalid DH public key")
        s = pow(peer_public, self._priv, _P)
        return int.from_bytes(hashlib.sha256(s.to_bytes(256, "big")).digest()[:16], "little")


class Masker:
    """One party's view of its pairwise mask streams."""

    def __init__(self, party: str, fxp_bits: int = 18):
        self.party = party
        self.fxp_bits = fxp_bits
        self._dh = DiffieHellman()
        self._gens: dict[str, L.PCG64] = {}   # peer -> generator at draw 0
        self._pos: dict[str, int] = {}        # peer -> draws consumed so far

    @property
    def public_key(self) -> int:
        return self._dh.public_key

    def agree(self, peer_keys: dict[str, int]) -> None:
        for peer, key in peer_keys.items():
            if peer != self.party:
                self.set_seed(peer, self._dh.shared_seed(key))

    def set_seed(self, peer: str, seed: int) -> None:
        self._gens[peer] = L.pcg64_from_seed(seed)
        self._pos[peer] = 0

    @property
    def peers(self) -> list[str]:
        return sorted(self._gens)

    def sign(self, peer: str) -> int:
        """+1: this party adds the pair mask (peer sorts after it), -1: subtracts."""
        return 1 if peer > self.party else -1

    def generator(self, peer: str, offset: int = 0) -> L.PCG64:
        """Generator positioned at the next unused draw (+ offset)."""
        return L.pcg64_advance(self._gens[peer], self._pos[peer] + offset)

    def streams(self, peers=None, offset: int = 0) -> list[tuple]:
        """(generator, sign, peer-index) triples for sa_mask."""
        peers = self.peers if peers is None else peers
        deltas = [self._pos[p] + offset for p in peers]
        if any(d >> 64 for d in deltas):
            gens = [self.generator(p, offset) for p in peers]
        else:  # one library call for every stream of the round
            gens = L.pcg64_advance_many([self._gens[p] for p in peers], deltas)
        return [(g, self.sign(p), i) for i, (g, p) in enumerate(zip(gens, peers))]

    def generators_at(self, peers) -> list:
        """The generators of ``peers`` at their next unused draws (one
        library call)."""
        return [g for g, _, _ in self.streams(peers)]

    def consume(self, n: int, peers=None) -> None:
        for p in (self.peers if peers is None else peers):
            self._pos[p] += int(n)

    def position(self, peer: str) -> int:
        return self._pos[peer]

    def skip(self, peer: str, k: int) -> None:
        """Raw draws consumed on top of one per element: numpy's
        Generator.integers rejected k raw outputs of 0 on this pair stream."""
        self._pos[peer] += int(k)

    def set_state(self, peer: str, state: int, inc: int) -> None:
        """Start the pair stream from an explicit numpy PCG64 (state, inc)
        (tests: a state whose next raw draws include a 0)."""
        self._gens[peer] = L.PCG64.of(int(state), int(inc))
        self._pos[peer] = 0

    def copy(self) -> "Masker":
        """An independent masker at the same stream positions (the per-party
        functions return a new masker each round).  The DH key pair and the
        draw-0 generators are never mutated in place -- ``set_seed`` /
        ``set_state`` replace dict entries -- so only the two dicts are
        copied (a ``copy.deepcopy`` of the ctypes generators took ~20 us a
        party, tools/latency_profile.py)."""
        m = object.__new__(Masker)
        m.party, m.fxp_bits, m._dh = self.party, self.fxp_bits, self._dh
        m._gens, m._pos = dict(self._gens), dict(self._pos)
        return m

    def snapshot(self) -> dict:
        return dict(self._pos)

    def restore(self, snap: dict) -> None:
        self._pos = dict(snap)
