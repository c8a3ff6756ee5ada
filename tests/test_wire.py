"""Wire format and loopback handshake (host logic, no GPU)."""
import socket
import threading

import numpy as np
import pytest

from sfl_amd import wire as W


def _pair():
    a, b = socket.socketpair()
    return a, b


def test_frame_roundtrip_u64_into_buffer():
    a, b = _pair()
    v = np.random.default_rng(0).integers(0, 2**64 - 1, 100_003, dtype=np.uint64)
    t = threading.Thread(target=W.send_frame, args=(a, W.MASKED, v), kwargs=dict(sender=3, rnd=7,
                                                                               digest=W.xor_digest(v)))
    t.start()
    buf = np.empty(100_003, dtype=np.int64)
    h, mv = W.recv_frame(b, into=buf, expect_kind=W.MASKED)
    t.join()
    assert (h.kind, h.dtype, h.sender, h.round, h.count, h.nbytes) == (W.MASKED, W.U64, 3, 7, 100_003, 800_024)
    assert np.array_equal(buf.view(np.uint64), v)
    assert h.digest == W.xor_digest(buf) == int(np.bitwise_xor.reduce(v))


@pytest.mark.parametrize("arr", [np.arange(5, dtype=np.float64), np.arange(7, dtype=np.float32), b"hello", None])
def test_frame_roundtrip_types(arr):
    a, b = _pair()
    W.send_frame(a, W.RESULT, arr)
    h, mv = W.recv_frame(b)
    if arr is None:
        assert h.count == 0 and len(mv) == 0
    elif isinstance(arr, bytes):
        assert bytes(mv) == arr and h.dtype == W.BYTES
    else:
        assert np.array_equal(W.as_array(h, mv), arr)


def test_header_validation():
    good = W.pack_header(W.MASKED, W.U64, 0, 0, 4)
    W.unpack_header(good)
    with pytest.raises(W.WireError, match="magic"):
        W.unpack_header(b"XXXX" + good[4:])
    with pytest.raises(W.WireError, match="version"):
        W.unpack_header(good[:4] + bytes([9]) + good[5:])
    bad = W.HEADER.pack(W.MAGIC, W.VERSION, W.MASKED, W.U64, 0, 0, 0, 4, 31, 0)
    with pytest.raises(W.WireError, match="inconsistent"):
        W.unpack_header(bad)
    with pytest.raises(W.WireError, match="short"):
        W.unpack_header(good[:10])


def test_truncated_frame_and_small_buffer():
    a, b = _pair()
    a.sendall(W.pack_header(W.MASKED, W.U64, 0, 0, 10) + b"\0" * 16)
    a.close()
    with pytest.raises(W.WireError, match="closed"):
        W.recv_frame(b)
    a, b = _pair()
    W.send_frame(a, W.MASKED, np.zeros(10, dtype=np.uint64))
    with pytest.raises(W.WireError, match="receive buffer"):
        W.recv_frame(b, into=np.empty(4, dtype=np.uint64))
    a, b = _pair()
    W.send_frame(a, W.KEYS, b"{}")
    with pytest.raises(W.WireError, match="expected frame kind"):
        W.recv_frame(b, expect_kind=W.MASKED)


def test_loopback_handshake_agrees_pair_seeds():
    """Server relays DH public keys; every pair of clients derives the same
    PCG64 generator (host-side C-ABI seeding, no GPU)."""
    from sfl_amd.loopback import LoopbackClient, LoopbackServer

    names = ["alice", "bob", "carol"]
    srv = LoopbackServer(len(names))
    clients = [None] * len(names)

    def run(i):
        c = LoopbackClient(names[i], i, srv.port)
        c.handshake()
        clients[i] = c

    ts = [threading.Thread(target=run, args=(i,)) for i in range(len(names))]
    for t in ts:
        t.start()
    keys = srv.accept(timeout=60)
    for t in ts:
        t.join()
    assert sorted(keys) == sorted(names) and srv.names == names
    for u in clients:
        for v in clients:
            if u is not v:
                gu, gv = u.masker.generator(v.party), v.masker.generator(u.party)
                assert (gu.state.lo, gu.state.hi, gu.inc.lo, gu.inc.hi) == (gv.state.lo, gv.state.hi, gv.inc.lo,
                                                                            gv.inc.hi)
                assert u.masker.sign(v.party) == -v.masker.sign(u.party)
    srv.close()
    for c in clients:
        c.close()


def test_chunked_receive_through_buffer_ring():
    a, b = _pair()
    v = np.random.default_rng(1).integers(0, 2**64 - 1, 10_007, dtype=np.uint64)
    t = threading.Thread(target=W.send_frame, args=(a, W.MASKED, v))
    t.start()
    h = W.recv_header(b, expect_kind=W.MASKED)
    ring = [np.empty(1000, dtype=np.uint64) for _ in range(2)]
    got = np.empty_like(v)
    seen = []

    def on_chunk(j, off, nbytes):
        got[off // 8: (off + nbytes) // 8] = ring[j][: nbytes // 8]
        seen.append((j, off, nbytes))

    W.recv_payload_chunked(b, h, ring, on_chunk)
    t.join()
    assert np.array_equal(got, v)
    assert [s[0] for s in seen] == [i % 2 for i in range(len(seen))] and len(seen) == 11


def test_oversized_control_frames_are_refused_before_allocation():
    """A peer announcing a huge HELLO / KEYS / META frame (the
    server read HELLO with an allocation sized by the peer's header) is
    refused at the header; unknown kinds too; RESULT frames respect the
    caller's expected size."""
    for kind in (W.HELLO, W.KEYS, W.META, W.BYE):
        hdr = W.pack_header(kind, W.BYTES, 0, 0, (1 << 20) + 1)
        with pytest.raises(W.WireError, match="control frame"):
            W.unpack_header(hdr)
        W.unpack_header(W.pack_header(kind, W.BYTES, 0, 0, 1 << 20))  # at the cap: fine
    with pytest.raises(W.WireError, match="unknown frame kind"):
        W.unpack_header(W.HEADER.pack(W.MAGIC, W.VERSION, 99, W.BYTES, 0, 0, 0, 4, 4, 0))
    a, b = _pair()
    a.sendall(W.pack_header(W.HELLO, W.BYTES, 0, 0, 1 << 39))  # 512 GiB claimed, nothing sent
    with pytest.raises(W.WireError, match="control frame"):
        W.recv_frame(b, expect_kind=W.HELLO)
    a, b = _pair()
    a.sendall(W.pack_header(W.RESULT, W.F64, 0, 0, 1 << 36))
    with pytest.raises(W.WireError, match="exceeds the expected"):
        W.recv_frame(b, expect_kind=W.RESULT, max_bytes=8 * 1000)
