"""The loopback runtime's send path (sfl_amd.loopback.SharedHostBuffer) on
the CPU, in both modes (sendall, and socket.sendfile of the memfd pages):
byte ranges sent over a socket with a
timeout (a non-blocking descriptor) whose buffer fills while the receiver
sleeps -- every byte arrives, in order, in several ranges.  (HIP registration
of the pages is exercised on the GPU by tests/test_gpu_loopback.py.)"""
import mmap
import os
import socket
import threading
import time

import numpy as np
import pytest

from sfl_amd import loopback as lb


class _Unregistered(lb.SharedHostBuffer):
    def __init__(self, nbytes):  # the memfd part only: no GPU here
        self.nbytes = nbytes
        self.fd = os.memfd_create("sfl_test")
        os.ftruncate(self.fd, nbytes)
        self._mm = mmap.mmap(self.fd, nbytes)
        self.array = np.frombuffer(self._mm, dtype=np.uint8)
        self.array[:] = np.arange(nbytes) % 251
        self._registered = False


@pytest.mark.parametrize("send", ["copy", "sendfile"])
def test_send_ranges_through_a_full_socket_buffer(monkeypatch, send):
    monkeypatch.setenv("SFL_LOOPBACK_SEND", send)
    n = 96 << 20
    buf = _Unregistered(n)
    srv = socket.create_server(("127.0.0.1", 0))
    got = bytearray(n)

    def rx():
        c, _ = srv.accept()
        c.settimeout(60)
        time.sleep(0.3)  # the sender's socket buffer fills meanwhile
        mv, k = memoryview(got), 0
        while k < n:
            r = c.recv_into(mv[k:])
            assert r
            k += r
        c.close()

    t = threading.Thread(target=rx)
    t.start()
    cs = socket.create_connection(("127.0.0.1", srv.getsockname()[1]), timeout=60)
    bounds = [0, 1, 4096, n // 3, n - 7, n]
    for lo, hi in zip(bounds, bounds[1:]):
        buf.send(cs, lo, hi)
    buf.send(cs, n, n)  # an empty range sends nothing
    t.join(60)
    cs.close()
    srv.close()
    assert bytes(got) == bytes(buf.array)
    buf.close()
    assert buf.fd == -1


def test_placement_one_process_per_gpu():
    """run_loopback(gpus=...): client process g on gpus[g % len(gpus)], the
    server on server_gpu (default gpus[0]) -- config 3 (8 processes on 8
    GPUs), config 5 (8 processes of 4 parties on 8 GPUs), the one-GPU boxes
    (gpus=[0, 0]) and more processes than GPUs."""
    assert lb.placement(8, list(range(8))) == (0, list(range(8)))
    assert lb.placement(8, list(range(8)), server_gpu=7) == (7, list(range(8)))
    assert lb.placement(3, [0, 0]) == (0, [0, 0, 0])
    assert lb.placement(5, [2, 3]) == (2, [2, 3, 2, 3, 2])
    assert lb.placement(0, [1]) == (1, [])
    with pytest.raises(ValueError):
        lb.placement(2, [])


def test_submit_failure_releases_the_result_receiver(monkeypatch):
    """a submit() that fails after its result-receiver thread
    started ends that thread (the connection is shut down) and clears the
    round in flight, so the failure is what the caller sees -- not a later
    'previous round's result was not collected'."""
    srv = socket.create_server(("127.0.0.1", 0))
    cl = lb.LoopbackClient("alice", 0, srv.getsockname()[1])
    peer, _ = srv.accept()

    def boom(*a, **k):
        raise RuntimeError("H2D failed")

    monkeypatch.setattr(cl, "_mask_and_send", boom)
    x = np.zeros(16, dtype=np.float32)
    with pytest.raises(RuntimeError, match="H2D failed"):
        cl.submit(x, 0, result_into=np.empty(16))
    assert cl._rx is None
    assert not [t for t in threading.enumerate() if getattr(t, "_target", None) == cl._receive_result]
    with pytest.raises(RuntimeError, match="H2D failed"):  # the same error again, not 'not collected'
        cl.submit(x, 1)
    cl.close()
    peer.close()
    srv.close()
