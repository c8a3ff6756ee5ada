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
