"""Framed raw wire format for masked vectors between party processes.

Replaces the RayFed ``.to(server)`` object transfer on the secure-aggregation
path (``sfl/distributed/op_strategy.py:131-141``) with a length-prefixed
binary frame whose payload is the raw little-endian array -- for masked
vectors plain uint64, the same scalar type the reference's interconnection
serializer carries (``SCALAR_TYPE_UINT64``, ``sfl/ic/proxy/serializer.py:263,335,359``)
but without per-element encoding, so a frame is sent and received with
zero copies (``sendall`` of the buffer, ``recv_into`` a pinned host buffer).

Frame = 48-byte header + payload::

    magic   4s  b"SFLW"
    version u8  1
    kind    u8  HELLO / KEYS / MASKED / RESULT / BYE / META
    dtype   u16 BYTES / U64 / F64 / F32
    sender  u32 party index
    rsvd    u32 0
    round   u64 aggregation round
    count   u64 elements
    nbytes  u64 payload bytes (= count * itemsize)
    digest  u64 XOR of the payload's u64 words (0 = not set)
"""

from __future__ import annotations

import socket
import struct
from typing import NamedTuple

import numpy as np

MAGIC = b"SFLW"
VERSION = 1
HEADER = struct.Struct("<4sBBHIIQQQQ")
assert HEADER.size == 48

HELLO, KEYS, MASKED, RESULT, BYE, META = 1, 2, 3, 4, 5, 6
BYTES, U64, F64, F32 = 0, 1, 2, 3
_ITEMSIZE = {BYTES: 1, U64: 8, F64: 8, F32: 4}
_NP = {U64: np.uint64, F64: np.float64, F32: np.float32}
MAX_FRAME_BYTES = 1 << 40
KINDS = (HELLO, KEYS, MASKED, RESULT, BYE, META)
# control frames (handshake, key table, per-round metadata, goodbye) are tiny:
# a peer announcing more is rejected before anything is allocated for it
CONTROL_KINDS = (HELLO, KEYS, META, BYE)
MAX_CONTROL_BYTES = 1 << 20


class WireError(RuntimeError):
    pass


class Header(NamedTuple):
    kind: int
    dtype: int
    sender: int
    round: int
    count: int
    nbytes: int
    digest: int


def dtype_code(a: np.ndarray) -> int:
    for code, t in _NP.items():
        if a.dtype == t:
            return code
    if a.dtype == np.int64:  # masked vectors carried as int64 bits
        return U64
    raise WireError(f"no wire type for {a.dtype}")


def xor_digest(buf) -> int:
    """XOR of the payload's 64-bit words (the kernels' masked-vector digest)."""
    v = np.frombuffer(buf, dtype=np.uint64)
    return int(np.bitwise_xor.reduce(v)) if v.size else 0


def pack_header(kind: int, dtype: int, sender: int, rnd: int, count: int, digest: int = 0) -> bytes:
    nbytes = count * _ITEMSIZE[dtype]
    return HEADER.pack(MAGIC, VERSION, kind, dtype, sender, 0, rnd, count, nbytes, digest)


def unpack_header(b: bytes) -> Header:
    if len(b) != HEADER.size:
        raise WireError(f"short header ({len(b)} bytes)")
    magic, ver, kind, dtype, sender, _r, rnd, count, nbytes, digest = HEADER.unpack(b)
    if magic != MAGIC:
        raise WireError(f"bad magic {magic!r}")
    if ver != VERSION:
        raise WireError(f"unsupported wire version {ver}")
    if dtype not in _ITEMSIZE:
        raise WireError(f"unknown dtype code {dtype}")
    if kind not in KINDS:
        raise WireError(f"unknown frame kind {kind}")
    if nbytes != count * _ITEMSIZE[dtype] or nbytes > MAX_FRAME_BYTES:
        raise WireError(f"inconsistent frame size: {count} x {_ITEMSIZE[dtype]} != {nbytes}")
    if kind in CONTROL_KINDS and nbytes > MAX_CONTROL_BYTES:
        raise WireError(f"control frame (kind {kind}) of {nbytes} bytes exceeds {MAX_CONTROL_BYTES}")
    return Header(kind, dtype, sender, rnd, count, nbytes, digest)


def recv_exact(sock: socket.socket, view: memoryview) -> None:
    """Fill ``view`` from the socket (raises WireError on a closed connection)."""
    _recv_exact(sock, view)


def _recv_exact(sock: socket.socket, view: memoryview) -> None:
    got = 0
    n = len(view)
    while got < n:
        k = sock.recv_into(view[got:], n - got)
        if k == 0:
            raise WireError(f"connection closed after {got} of {n} bytes")
        got += k


def send_frame(sock: socket.socket, kind: int, payload=None, *, dtype: int | None = None, sender: int = 0,
               rnd: int = 0, digest: int = 0) -> None:
    """Send one frame.  ``payload``: bytes, a numpy array, or a CPU torch
    tensor (sent from its memory, no copy)."""
    if payload is None:
        mv = memoryview(b"")
        dtype = BYTES if dtype is None else dtype
    elif isinstance(payload, (bytes, bytearray, memoryview)):
        mv = memoryview(payload).cast("B")
        dtype = BYTES if dtype is None else dtype
    else:
        a = payload.numpy() if hasattr(payload, "numpy") and not isinstance(payload, np.ndarray) else payload
        a = np.ascontiguousarray(a)
        dtype = dtype_code(a) if dtype is None else dtype
        mv = memoryview(a).cast("B")
    isz = _ITEMSIZE[dtype]
    if len(mv) % isz:
        raise WireError(f"payload of {len(mv)} bytes is not a whole number of {isz}-byte elements")
    sock.sendall(pack_header(kind, dtype, sender, rnd, len(mv) // isz, digest))
    if len(mv):
        sock.sendall(mv)


def recv_header(sock: socket.socket, *, expect_kind: int | None = None) -> Header:
    hb = bytearray(HEADER.size)
    _recv_exact(sock, memoryview(hb))
    h = unpack_header(bytes(hb))
    if expect_kind is not None and h.kind != expect_kind:
        raise WireError(f"expected frame kind {expect_kind}, got {h.kind}")
    return h


def recv_payload_chunked(sock: socket.socket, h: Header, buffers, on_chunk) -> None:
    """Stream a frame's payload through a ring of host buffers (numpy arrays
    or pinned CPU tensors): chunk j lands in buffers[j % len(buffers)], then
    ``on_chunk(buf_index, byte_offset, nbytes)`` runs; the callback owns
    waiting until a buffer is free again before returning."""
    views = [memoryview(b.numpy() if hasattr(b, "numpy") and not isinstance(b, np.ndarray) else b).cast("B")
             for b in buffers]
    cap = min(len(v) for v in views)
    off, j = 0, 0
    while off < h.nbytes:
        k = min(cap, h.nbytes - off)
        _recv_exact(sock, views[j % len(views)][:k])
        on_chunk(j % len(views), off, k)
        off += k
        j += 1


def recv_frame(sock: socket.socket, into=None, *, expect_kind: int | None = None, max_bytes: int | None = None):
    """Receive one frame -> (Header, memoryview of the payload).  With
    ``into`` (a writable buffer: numpy array / pinned CPU tensor), the payload
    lands there directly and must fit; otherwise a buffer of the announced
    size is allocated, which must not exceed ``max_bytes`` when given
    (control frames are capped at MAX_CONTROL_BYTES by the header check)."""
    h = recv_header(sock, expect_kind=expect_kind)
    if into is None and max_bytes is not None and h.nbytes > max_bytes:
        raise WireError(f"frame payload of {h.nbytes} bytes exceeds the expected {max_bytes}")
    if into is not None:
        a = into.numpy() if hasattr(into, "numpy") and not isinstance(into, np.ndarray) else into
        mv = memoryview(a).cast("B")
        if len(mv) < h.nbytes:
            raise WireError(f"receive buffer of {len(mv)} bytes < frame payload {h.nbytes}")
        mv = mv[:h.nbytes]
    else:
        mv = memoryview(bytearray(h.nbytes))
    _recv_exact(sock, mv)
    return h, mv


def as_array(h: Header, mv: memoryview) -> np.ndarray:
    if h.dtype == BYTES:
        return np.frombuffer(mv, dtype=np.uint8)
    return np.frombuffer(mv, dtype=_NP[h.dtype])
