"""Loopback-socket party runtime for secure aggregation.

Every party is its own OS process; parties talk only through TCP sockets on
127.0.0.1 using the framed raw wire format (``sfl_amd.wire``), replacing the
RayFed actor transport of the reference (``sfl/distributed/op_strategy.py:131-141``):

1. handshake -- each client sends HELLO (party name, index, DH public key);
   the server relays the key table (KEYS) and every client derives its
   pairwise seeds (``Masker.agree``, the a1 setup of SURVEY.md §8a);
2. round -- each client copies its host gradient to its GPU, quantizes and
   masks it there (``sa_mask``), copies the masked uint64 vector back to
   pinned host memory and sends it (META with its weight, then MASKED); the
   server receives all C frames concurrently straight into pinned buffers
   and copies each chunk to its GPU as it lands; as soon as a chunk of every
   client is there it sums those slices mod 2^64 (``sa_sum_u64``), decodes
   them (``sa_decode``) and streams that chunk of the float64 result back
   to every client (RESULT) while later chunks are still arriving.

This is the path that "starts and ends in host memory" (BASELINE north
star): the per-round rate here includes H2D, D2H and the loopback copies.
The GPU kernels are the product path; nothing here falls back to the CPU.

Host buffers that leave through a socket (every client's masked vector, the
server's float64 result) are ``SharedHostBuffer``s: memfd-backed pages that
are HIP-registered, so the D2H copy lands in them directly.  They are sent
with ``sendall`` (a copy into the kernel); ``SFL_LOOPBACK_SEND=sendfile``
hands the page references to the socket instead -- no send-side copy, but
measured no faster at 8 x 100M and slower at 32 x 256M (DESIGN.md §7,
tools/socket_floor.py for the transport alone).  Clients receive the result
while they send, and GPU waits poll instead of spinning a core.
"""

from __future__ import annotations

import json
import os
import socket
import threading
import time
from collections import defaultdict
from contextlib import contextmanager

import numpy as np

from . import hostpipe as H
from . import wire as W
from .wire import META

CHUNK_ELEMS = 8 << 20  # 64 MiB of u64 per pinned staging buffer


class StageClock:
    """Wall and thread-CPU seconds (user + system, so the kernel's socket
    copies count) per named stage of a round, summed over the threads that
    ran it: the host-side profile of the loopback path
    (tools/loopback_bench.py --stages)."""

    def __init__(self):
        self._t = defaultdict(lambda: [0.0, 0.0, 0])
        self._lock = threading.Lock()

    @contextmanager
    def __call__(self, name: str):
        w0, c0 = time.perf_counter(), time.thread_time()
        try:
            yield
        finally:
            w, c = time.perf_counter() - w0, time.thread_time() - c0
            with self._lock:
                e = self._t[name]
                e[0] += w
                e[1] += c
                e[2] += 1

    def report(self) -> dict:
        with self._lock:
            return {k: {"wall_s": v[0], "cpu_s": v[1], "calls": v[2]} for k, v in sorted(self._t.items())}


# Knobs for same-box A/B measurements of the host path (tools/loopback_bench.py
# --ab); the defaults are the product's choices.
#   SFL_LOOPBACK_SEND=copy|sendfile   sendall() (a copy into the kernel), or sendfile() from the memfd pages
#                                     (no send-side copy, but page-granular kernel work: measured no faster
#                                     at 8 x 100M and 26 % slower at 32 x 256M, profiles/r03/loopback_*_ab.jsonl)
#   SFL_LOOPBACK_WAIT=poll|spin       wait for a GPU event by polling with short sleeps, or in hipEventSynchronize
#   SFL_LOOPBACK_CLIENT_RX=concurrent|after   a client reads the result while it sends, or after (round 2;
#                                     with SEND=sendfile that can stall on the box's kernel: copy only)
def _send_mode() -> str:
    return os.environ.get("SFL_LOOPBACK_SEND", "copy")


def wait_event(e) -> None:
    """Wait for a recorded GPU event.  hipEventSynchronize spins a CPU core
    for the whole wait; the loopback party runs ~20 threads per process
    against the box's CPU share, so a wait polls with ~50 us sleeps instead
    and leaves the core to the socket copies."""
    if os.environ.get("SFL_LOOPBACK_WAIT", "poll") == "spin":
        e.synchronize()
        return
    while not e.query():
        time.sleep(50e-6)


_HIP = None


def _hip():
    global _HIP
    if _HIP is None:
        import ctypes

        _HIP = ctypes.CDLL("libamdhip64.so")
    return _HIP


class SharedHostBuffer:
    """``nbytes`` of memfd-backed host memory, mapped, faulted in and
    HIP-registered (hipHostRegister): device copies land in it directly (torch
    sees it as pinned), and ``send(sock, lo, hi)`` ships a byte range --
    with ``sendall``, or with ``os.sendfile`` (page references handed to the
    socket, no send-side copy) under SFL_LOOPBACK_SEND=sendfile.  With
    sendfile the pages must not change until the peer has read them; the
    round protocol guarantees that (a party writes a buffer again only after
    every peer answered the frame that carried it)."""

    def __init__(self, nbytes: int, dtype=np.float64):
        import ctypes
        import mmap

        self.nbytes = max(int(nbytes), 8)
        self.fd = os.memfd_create("sfl_sa_wire", os.MFD_CLOEXEC)
        try:
            os.ftruncate(self.fd, self.nbytes)
            self._mm = mmap.mmap(self.fd, self.nbytes)
        except BaseException:
            os.close(self.fd)
            raise
        self.array = np.frombuffer(self._mm, dtype=dtype)
        self.array.view(np.uint8)[:] = 0  # fault every page in before registering
        self._ptr = self.array.ctypes.data
        rc = _hip().hipHostRegister(ctypes.c_void_p(self._ptr), ctypes.c_size_t(self.nbytes), ctypes.c_uint(0))
        if rc != 0:
            self._close_map()
            raise RuntimeError(f"hipHostRegister of a {self.nbytes}-byte memfd buffer failed (hipError {rc})")
        self._registered = True

    def tensor(self):
        import torch

        return torch.from_numpy(self.array)

    def send(self, sock: socket.socket, lo: int, hi: int) -> None:
        """Send bytes [lo, hi) of the buffer (socket.sendfile: os.sendfile
        plus the wait for a full socket buffer that a socket with a timeout,
        i.e. a non-blocking descriptor, needs)."""
        if hi <= lo:
            return
        if _send_mode() == "copy":
            sock.sendall(memoryview(self.array).cast("B")[lo:hi])
            return
        f = open(self.fd, "rb", buffering=0, closefd=False)  # a file object on the memfd (no new open)
        try:
            sent = sock.sendfile(f, lo, hi - lo)
        finally:
            f.close()
        if sent != hi - lo:
            raise W.WireError(f"sendfile sent {sent} of {hi - lo} bytes (peer closed?)")

    def _close_map(self):
        self.array = None
        try:
            self._mm.close()
        except BufferError:  # a view of the pages is still alive: the mapping goes with it
            pass
        os.close(self.fd)
        self.fd = -1

    def close(self):
        if getattr(self, "_registered", False):
            import ctypes

            _hip().hipHostUnregister(ctypes.c_void_p(self._ptr))
            self._registered = False
        if getattr(self, "fd", -1) >= 0:
            self._close_map()

    def __del__(self):
        try:
            self.close()
        except Exception:  # noqa: BLE001 - interpreter shutdown
            pass


def chunk_elems() -> int:
    """Staging chunk (elements); SFL_LOOPBACK_CHUNK_ELEMS overrides (tests)."""
    return int(os.environ.get("SFL_LOOPBACK_CHUNK_ELEMS", CHUNK_ELEMS))


class LoopbackServer:
    """The aggregation server party (binds 127.0.0.1)."""

    def __init__(self, n_clients: int, *, host: str = "127.0.0.1", port: int = 0, gpu: int = 0,
                 fxp_bits: int = 18):
        self.n_clients = n_clients
        self.gpu = gpu
        self.fxp_bits = fxp_bits
        self.sock = socket.create_server((host, port))
        self.port = self.sock.getsockname()[1]
        self.conns: list[socket.socket] = []
        self.names: list[str] = []
        self._bufs = None
        self.last_masked = None

    def accept(self, timeout: float = 300.0) -> dict:
        """Accept every client, collect HELLOs, relay the key table."""
        self.sock.settimeout(timeout)
        hello = {}
        for _ in range(self.n_clients):
            conn, _ = self.sock.accept()
            conn.settimeout(timeout)
            conn.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            _, mv = W.recv_frame(conn, expect_kind=W.HELLO)
            info = json.loads(bytes(mv))
            hello[int(info["index"])] = (conn, info)
        if sorted(hello) != list(range(self.n_clients)):
            raise W.WireError(f"client indices {sorted(hello)} are not 0..{self.n_clients - 1}")
        self.conns = [hello[i][0] for i in range(self.n_clients)]
        self.names = [hello[i][1]["party"] for i in range(self.n_clients)]
        if len(set(self.names)) != len(self.names):
            raise W.WireError(f"duplicate party names {self.names}")
        keys = {hello[i][1]["party"]: hello[i][1]["public_key"] for i in range(self.n_clients)}
        blob = json.dumps(keys).encode()
        for c in self.conns:
            W.send_frame(c, W.KEYS, blob)
        return keys

    def _buffers(self, n: int):
        import torch

        if self._bufs is None or self._bufs[0] != n:
            dev = torch.device("cuda", self.gpu)
            ce = min(n, chunk_elems())
            if self._bufs is not None:  # the old result pages (8n bytes, HIP-registered) go now, not at GC
                self._bufs[4][2].close()
                self._bufs = None
            ring = [[torch.empty(ce, dtype=torch.int64).pin_memory() for _ in range(2)] for _ in self.conns]
            devb = [torch.empty(n, dtype=torch.int64, device=dev) for _ in self.conns]
            streams = [torch.cuda.Stream(dev) for _ in self.conns]
            # the float64 result: D2H straight into the registered pages the broadcast sends
            agg = (torch.empty(n, dtype=torch.int64, device=dev), torch.empty(n, dtype=torch.float64, device=dev),
                   SharedHostBuffer(8 * n, np.float64), torch.cuda.Stream(dev))
            self._bufs = (n, ring, devb, streams, agg)
        return self._bufs[1:]

    def round(self, n: int, rnd: int, **kw):
        """One aggregation round on the server's GPU (``_round``): HIP calls
        made here without a tensor argument (host registration, events) go
        to that device too, whatever device the calling process is on."""
        import torch

        with torch.cuda.device(self.gpu):
            return self._round(n, rnd, **kw)

    def _round(self, n: int, rnd: int, *, average: bool = False, verify_digest: bool = False,
               keep_masked: bool = False, timeout: float = 600.0, copy_out: bool = True):
        """One aggregation round over n-element vectors -> (float64 result, timings).

        ``copy_out=False`` returns the server's own result buffer (the pages the
        broadcast sent) instead of a copy: valid until the next round().

        Pipelined per chunk (chunk_elems() elements): every connection's frame
        streams through a ring of two pinned buffers and each chunk is copied
        to the device as it lands (one stream per client); as soon as chunk j
        of EVERY client is on the device, the server sums those slices mod
        2^64, decodes them and copies the float64 chunk to pinned host memory
        (its own stream), and one sender thread per client streams the RESULT
        frame chunk by chunk -- so the broadcast of early chunks overlaps the
        reception of later ones and host memory stays O(chunk) per client."""
        import threading

        import torch

        from . import kernels as K

        ring, devb, streams, (s_sum, dec, res_shb, agg) = self._buffers(n)
        res_host = res_shb.tensor()
        C = len(self.conns)
        ce = ring[0][0].numel()
        bounds = [(lo, min(n, lo + ce)) for lo in range(0, n, ce)] or [(0, 0)]
        J = len(bounds)
        t0 = time.perf_counter()
        weights = [None] * C
        arrived = [0] * J
        ev_in = [[None] * J for _ in range(C)]
        cond = threading.Condition()
        errors = []
        done_rx = [0]  # receivers finished (an empty frame has no chunks)
        ready = [threading.Event() for _ in range(J)]
        stamps = {}
        clock = StageClock()

        def receive(i):
            try:
                conn = self.conns[i]
                _, mv = W.recv_frame(conn, expect_kind=META)
                weights[i] = json.loads(bytes(mv)).get("weight")
                h = W.recv_header(conn, expect_kind=W.MASKED)
                if h.count != n or h.round != rnd or h.dtype != W.U64:
                    raise W.WireError(f"client {i}: frame of {h.count} elems for round {h.round}, want {n} / {rnd}")
                events = [None, None]
                dig = [0]

                def on_chunk(b, off, nbytes):
                    k, e0 = nbytes // 8, off // 8
                    if verify_digest:
                        dig[0] ^= W.xor_digest(ring[i][b].numpy()[:k])
                    with clock("server: H2D enqueue (pinned ring -> GPU)"):
                        with torch.cuda.stream(streams[i]):
                            devb[i][e0:e0 + k].copy_(ring[i][b][:k], non_blocking=True)
                            events[b] = torch.cuda.Event()
                            events[b].record(streams[i])
                    with cond:
                        j = e0 // ce
                        ev_in[i][j] = events[b]
                        arrived[j] += 1
                        cond.notify_all()
                    if events[1 - b] is not None:  # the other buffer is received into next
                        with clock("server: wait for the ring buffer's H2D"):
                            wait_event(events[1 - b])

                with clock("server: receive thread total (socket recv_into the pinned ring + the above)"):
                    W.recv_payload_chunked(conn, h, ring[i], on_chunk)
                if verify_digest and h.digest != dig[0]:
                    raise W.WireError(f"client {i}: payload digest mismatch")
                with cond:
                    done_rx[0] += 1
                    cond.notify_all()
            except BaseException as e:  # noqa: BLE001 - reported by the coordinator
                with cond:
                    errors.append(e)
                    cond.notify_all()

        def send(i):
            try:
                conn = self.conns[i]
                conn.sendall(W.pack_header(W.RESULT, W.F64, 0, rnd, n))
                for j, (lo, hi) in enumerate(bounds):
                    with clock("server: send thread waits for a result chunk"):
                        if not ready[j].wait(timeout):
                            raise TimeoutError(f"result chunk {j} not ready")
                    if errors:
                        return
                    if hi > lo:
                        with clock("server: broadcast send (result pages -> socket)"):
                            res_shb.send(conn, 8 * lo, 8 * hi)
            except BaseException as e:  # noqa: BLE001
                with cond:
                    errors.append(e)
                    cond.notify_all()

        res_np = res_shb.array[:n]
        out = np.empty(n, dtype=np.float64) if copy_out else res_np  # the caller's copy, filled chunk by chunk
        rx = [threading.Thread(target=receive, args=(i,), daemon=True) for i in range(C)]
        tx = [threading.Thread(target=send, args=(i,), daemon=True) for i in range(C)]
        for t in rx + tx:
            t.start()
        try:
            div = None
            for j, (lo, hi) in enumerate(bounds):
                with clock("server: wait for chunk j of every client"), cond:
                    if not cond.wait_for(lambda: errors or arrived[j] == C or done_rx[0] == C, timeout):
                        raise TimeoutError(f"chunk {j} not received from every client")
                    if errors:
                        raise errors[0]
                if j == 0:
                    stamps["first_chunk_all"] = time.perf_counter()
                if div is None:
                    div = 1.0
                    if average:
                        div = float(C) if all(w is None for w in weights) else float(
                            sum(1.0 if w is None else w for w in weights))
                with torch.cuda.stream(agg):
                    for i in range(C):
                        if ev_in[i][j] is not None:
                            agg.wait_event(ev_in[i][j])
                    if hi > lo:
                        K.sum_u64([d[lo:hi] for d in devb], s_sum[lo:hi])
                        K.decode(s_sum[lo:hi], dec[lo:hi], fxp_bits=self.fxp_bits, divisor=div)
                        res_host[lo:hi].copy_(dec[lo:hi], non_blocking=True)
                    e = torch.cuda.Event()
                    e.record(agg)
                with clock("server: sum + decode + D2H of the chunk (GPU)"):
                    wait_event(e)
                ready[j].set()
                # copy the chunk out of the result pages while it is broadcast
                # and later chunks arrive (no 8n-byte copy after the round)
                if copy_out:
                    with clock("server: copy-out (result pages -> caller's array, memcpy)"):
                        out[lo:hi] = res_np[lo:hi]
            stamps["recv_done"] = time.perf_counter()
            for t in rx + tx:
                t.join(timeout)
            if errors:
                raise errors[0]
            if any(t.is_alive() for t in rx + tx):
                raise TimeoutError("a party's receive or result send did not finish")
        except BaseException as e:
            with cond:  # senders released below must see the failure and send nothing more
                if e not in errors:
                    errors.append(e)
            raise
        finally:
            for r in ready:  # release senders (on an error they stop before sending)
                r.set()
        t_end = time.perf_counter()
        if keep_masked:
            for st in streams:
                st.synchronize()
            self.last_masked = [H.d2h(d, pooled=False).view(np.uint64) for d in devb]
        return out, {"first_chunk_all_s": stamps["first_chunk_all"] - t0,
                     "recv_sum_decode_s": stamps["recv_done"] - t0,
                     "broadcast_tail_s": t_end - stamps["recv_done"],
                     "round_s": t_end - t0, "chunks": J, "stages": clock.report()}

    def close(self):
        for c in self.conns:
            try:
                W.send_frame(c, W.BYE)
                c.close()
            except OSError:
                pass
        self.sock.close()
        if self._bufs is not None:
            self._bufs[4][2].close()
            self._bufs = None


class LoopbackClient:
    """One client party: masks its host vector on its GPU and ships it."""

    def __init__(self, party: str, index: int, port: int, *, host: str = "127.0.0.1", gpu: int = 0,
                 fxp_bits: int = 18, seeds: dict | None = None):
        from .security.aggregation.masker import Masker

        self.party, self.index, self.gpu = party, index, gpu
        self.masker = Masker(party, fxp_bits)
        self.fxp_bits = fxp_bits
        self._seeds = seeds
        self.sock = socket.create_connection((host, port), timeout=300)
        self.sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        self._bufs = None
        self._rx = None  # the result receiver of the round in flight (submit(result_into=...))

    def handshake(self):
        hello = {"party": self.party, "index": self.index, "public_key": self.masker.public_key}
        W.send_frame(self.sock, W.HELLO, json.dumps(hello).encode(), sender=self.index)
        _, mv = W.recv_frame(self.sock, expect_kind=W.KEYS)
        keys = {k: int(v) for k, v in json.loads(bytes(mv)).items()}
        if self._seeds is not None:  # explicit pair seeds (tests / benches)
            for peer in keys:
                if peer != self.party:
                    sd = self._seeds[peer]
                    if isinstance(sd, (tuple, list)):  # explicit numpy PCG64 (state, inc)
                        self.masker.set_state(peer, *sd)
                    else:
                        self.masker.set_seed(peer, int(sd))
        else:
            self.masker.agree(keys)
        return sorted(keys)

    def _buffers(self, n: int):
        import torch

        if self._bufs is None or self._bufs[0] != n:
            dev = torch.device("cuda", self.gpu)
            ce = min(n, chunk_elems())
            if self._bufs is not None:
                self._bufs[2].close()
            # the masked vector: D2H straight into registered pages, sent chunk by chunk
            self._bufs = (n, [torch.empty(ce, dtype=torch.float32).pin_memory() for _ in range(2)],
                          SharedHostBuffer(8 * n, np.int64),
                          torch.empty(n, dtype=torch.float32, device=dev),
                          torch.empty(n, dtype=torch.int64, device=dev), torch.cuda.Stream(dev))
        return self._bufs[1:]

    def _receive_result(self, n, into, box):
        """The RESULT frame, chunk by chunk: into ``into`` (n elements) or,
        when ``into`` is a list of two chunk buffers, through that ring (the
        caller keeps only the checksum); the XOR of its 64-bit words is
        folded in as each chunk lands (``box["xor"]``)."""
        try:
            w0, c0 = time.perf_counter(), time.thread_time()
            h = W.recv_header(self.sock, expect_kind=W.RESULT)
            if h.dtype != W.F64 or h.count != int(n):
                raise W.WireError(f"RESULT frame of {h.count} elements (dtype {h.dtype}), want {n} float64")
            ring = isinstance(into, list)
            ce = into[0].size if ring else chunk_elems()
            x, j = 0, 0
            for lo in range(0, n, ce):
                k = min(ce, n - lo)
                buf = into[j & 1][:k] if ring else into[lo:lo + k]
                W.recv_exact(self.sock, memoryview(buf).cast("B"))
                x ^= int(np.bitwise_xor.reduce(buf.view(np.uint64))) if k else 0
                j += 1
            box["h"], box["xor"] = h, x
            self.last_result_recv = {"wall_s": time.perf_counter() - w0, "cpu_s": time.thread_time() - c0}
        except BaseException as e:  # noqa: BLE001 - re-raised by result()
            box["error"] = e

    def submit(self, x: np.ndarray, rnd: int, weight=None, dp=None, result_into: np.ndarray | None = None) -> dict:
        """Mask ``x`` (host float32) for round ``rnd`` and send it.  With a
        ``GaussianModelDP`` ``dp``, its clip + noise runs inside the masking
        kernel (``sa_mask_dp``) on the device copy of ``x``.  ``x`` streams to
        the device through two pinned chunk buffers; the masked vector comes
        back chunk by chunk into registered memfd pages, each chunk sent as it
        lands.

        ``result_into`` (float64, n elements; or a list of two float64 chunk
        buffers when only the checksum is wanted): the round's RESULT frame is
        received into it by a thread started now, while this party is still
        sending -- the server broadcasts chunk j as soon as it has chunk j of
        every party, and a party that read only after sending everything
        would leave both directions of its connection full at once (on the
        GPU box's kernel that stalls sendfile()d transfers, tools/socket_floor.py
        --client-sequential).  ``result()`` then joins it; ``last_result_xor``
        holds the XOR of the result's 64-bit words."""
        n = x.size
        if self._rx is not None:
            raise RuntimeError("the previous round's result was not collected (result())")
        if result_into is not None:
            bufs = result_into if isinstance(result_into, list) else [result_into]
            for b in bufs:
                if b.dtype != np.float64 or not b.flags.c_contiguous:
                    raise ValueError("result_into: contiguous float64 arrays")
            if isinstance(result_into, list):
                if len(result_into) != 2 or min(b.size for b in result_into) < 1:
                    raise ValueError("result_into: a ring of two chunk buffers")
                target, keep = result_into, None
            else:
                if result_into.size < n:
                    raise ValueError("result_into must hold at least n elements")
                target = keep = result_into[:n]
            box = {}
            t = threading.Thread(target=self._receive_result, args=(n, target, box), daemon=True)
            t.start()
            self._rx = (t, box, keep, n)
        try:
            return self._mask_and_send(x, n, rnd, weight, dp)
        except BaseException:
            # the result receiver started above would stay blocked in recv and
            # the next submit() would report an uncollected round: end the
            # connection (the server sees the failure) and the thread with it
            if self._rx is not None:
                t = self._rx[0]
                self._rx = None
                try:
                    self.sock.shutdown(socket.SHUT_RDWR)
                except OSError:
                    pass
                t.join(timeout=30)
            raise

    def _mask_and_send(self, x: np.ndarray, n: int, rnd: int, weight, dp) -> dict:
        import torch

        from . import _lib as L
        from . import kernels as K

        hx, hmb, dx, dm, cs = self._buffers(n)
        hm = hmb.tensor()
        dev = dx.device
        ce = hx[0].numel()
        xf = np.asarray(x, dtype=np.float32).reshape(-1)
        clock = StageClock()
        t0 = time.perf_counter()
        ev = [None, None]
        with torch.cuda.stream(cs):
            for j, lo in enumerate(range(0, n, ce)):
                b, k = j & 1, min(ce, n - lo)
                if ev[b] is not None:
                    with clock("client: wait for the staging buffer's H2D"):
                        wait_event(ev[b])
                with clock("client: stage in (numpy -> pinned, memcpy)"):
                    hx[b].numpy()[:k] = xf[lo:lo + k]
                dx[lo:lo + k].copy_(hx[b][:k], non_blocking=True)
                ev[b] = torch.cuda.Event()
                ev[b].record(cs)
            dig = torch.zeros(1, dtype=torch.int64, device=dev)
            flags = torch.zeros(1, dtype=torch.int32, device=dev)
            w = 1.0 if weight is None else weight
            if dp is None:
                K.mask(dx, dm, self.masker.streams(), weight=w, fxp_bits=self.fxp_bits, digest=dig, flags=flags)
            else:  # clip + noise inside the masking kernel (sa_mask_dp; tools/dp_bench.py)
                K.mask_dp(dx, dm, self.masker.streams(), dp.params(dp.sumsq([dx]), n), weight=w,
                          fxp_bits=self.fxp_bits, digest=dig, flags=flags)
        with clock("client: last H2D + mask kernel (GPU)"):
            cs.synchronize()
        extra = {}
        if int(flags.item()) & L.SA_FLAG_PRG_REJECT:
            # numpy's Generator.integers rejected a raw 0 on some stream: move
            # the masked vector onto numpy's stream from there (sa_stream_shift)
            with torch.cuda.stream(cs):
                streams = self.masker.streams()
                found = K.rejected_draws_many([g for g, _, _ in streams], n, dev)
                for peer, (gen, sign, _), (pts, total) in zip(self.masker.peers, streams, found):
                    for k, shift in pts:
                        K.stream_shift(dm, gen, sign, k, shift)
                    if total > n:
                        extra[peer] = total - n
                dig.zero_()
                K.xor_digest(dm, dig)
            cs.synchronize()
        self.masker.consume(n)
        for peer, k in extra.items():
            self.masker.skip(peer, k)
        t1 = time.perf_counter()
        W.send_frame(self.sock, META, json.dumps({"weight": weight}).encode(), sender=self.index, rnd=rnd)
        self.sock.sendall(W.pack_header(W.MASKED, W.U64, self.index, rnd, n,
                                        int(dig.cpu().numpy().view(np.uint64)[0])))
        # every chunk's D2H enqueued at once (each lands in its own pages);
        # a chunk is sent as soon as its copy has finished
        chunks = []
        with torch.cuda.stream(cs):
            for lo in range(0, n, ce):
                hi = min(n, lo + ce)
                hm[lo:hi].copy_(dm[lo:hi], non_blocking=True)
                e = torch.cuda.Event()
                e.record(cs)
                chunks.append((lo, hi, e))
        for lo, hi, e in chunks:
            with clock("client: wait for a chunk's D2H"):
                wait_event(e)
            with clock("client: send (masked-vector pages -> socket)"):
                hmb.send(self.sock, 8 * lo, 8 * hi)
        t2 = time.perf_counter()
        self.last_stages = clock.report()
        return {"h2d_mask_s": t1 - t0, "d2h_send_s": t2 - t1, "stages": self.last_stages}

    def result(self, n: int | None = None, into: np.ndarray | None = None) -> np.ndarray:
        """The server's float64 aggregate (``n`` elements when given: a larger
        announced frame is refused before anything is allocated).  The
        payload is received straight into the returned array -- ``into``
        (float64, reused across rounds by a caller that consumes each result
        before the next) or a fresh one -- with no intermediate copy."""
        if self._rx is not None:  # received concurrently with submit(result_into=...)
            t, box, buf, rn = self._rx
            self._rx = None
            t.join()
            if "error" in box:
                raise box["error"]
            if n is not None and int(n) != rn:
                raise W.WireError(f"RESULT of {rn} elements, want {n}")
            self.last_result_xor = box["xor"]
            return buf
        if into is None and n is not None:
            into = np.empty(int(n), dtype=np.float64)
        if into is None:
            h, mv = W.recv_frame(self.sock, expect_kind=W.RESULT)
            return W.as_array(h, mv).copy()
        if isinstance(into, list):  # a ring of two chunk buffers: the checksum only
            if n is None:
                raise ValueError("a result ring needs n")
            box = {}
            self._receive_result(int(n), into, box)
            if "error" in box:
                raise box["error"]
            self.last_result_xor = box["xor"]
            return None
        if into.dtype != np.float64 or not into.flags.c_contiguous:
            raise ValueError("result buffer must be a contiguous float64 array")
        if n is not None:
            box = {}
            self._receive_result(int(n), into[:int(n)], box)
            if "error" in box:
                raise box["error"]
            self.last_result_xor = box["xor"]
            return into[:int(n)]
        w0, c0 = time.perf_counter(), time.thread_time()
        h, _ = W.recv_frame(self.sock, into, expect_kind=W.RESULT)
        self.last_result_recv = {"wall_s": time.perf_counter() - w0, "cpu_s": time.thread_time() - c0}
        if h.dtype != W.F64:
            raise W.WireError(f"RESULT frame of dtype {h.dtype}, want float64")
        return into[:h.count]

    def close(self):
        try:
            self.sock.close()
        except OSError:
            pass
        if self._bufs is not None:
            self._bufs[2].close()
            self._bufs = None


# ---------------------------------------------------------------------------
# process orchestration (spawned client processes, server in the caller)
# ---------------------------------------------------------------------------
def synthetic_gradient(c: int, n: int, rnd: int = 0) -> np.ndarray:
    """SURVEY.md §8(d) synthetic input: N(0, 0.01^2) float32, seeded per client."""
    g = np.random.default_rng(20260116 + c + 1000 * rnd)
    return (g.standard_normal(n, dtype=np.float32) * np.float32(1e-2)).astype(np.float32)


def placement(n_procs: int, gpus: list[int], server_gpu: int | None = None) -> tuple[int, list[int]]:
    """Where the parties run: (the server's GPU, the GPU of each client
    process g = gpus[g % len(gpus)]).  One client process per GPU on the
    8-GPU node (config 3), or four parties per process and one process per
    GPU (config 5), so every GPU's PCIe link carries only its own parties'
    H2D / D2H -- as the reference runs one party per process on its own
    device (tests/conftest.py:386-394, sfl/distributed/op_strategy.py:131-141).
    The server takes ``server_gpu`` (default ``gpus[0]``)."""
    if not gpus:
        raise ValueError("placement: no GPUs")
    if n_procs < 0:
        raise ValueError("placement: negative process count")
    return (gpus[0] if server_gpu is None else server_gpu), [gpus[g % len(gpus)] for g in range(n_procs)]


def client_process(parties: list, port: int, n: int, rounds: int, gpu: int, fxp_bits: int, out_q,
                   keep_results: bool = True) -> None:
    """Entry point of one spawned process hosting one or more client parties
    (``parties``: (name, index, pair seeds or None, weight) tuples), each on
    its own socket and thread, all on GPU ``gpu``.  Every party records the
    XOR of each round's result; ``keep_results=False`` receives the results
    through a ring of two chunk buffers instead of a whole-vector array
    (config 5's 32 parties x 256M elements would otherwise hold 64 GB of
    results)."""
    import threading

    import torch

    torch.cuda.set_device(gpu)  # this process's HIP calls (host registration, copies) on its own GPU
    dump_after = float(os.environ.get("SFL_LOOPBACK_DUMP_AFTER", "0"))
    if dump_after > 0:  # diagnostics: every thread's stack if the process is still here then
        import faulthandler

        faulthandler.dump_traceback_later(dump_after, exit=False)

    def run(party, index, seeds, weight):
        try:
            xs = [synthetic_gradient(index, n, r) for r in range(rounds)]  # generated outside the rounds
            cl = LoopbackClient(party, index, port, gpu=gpu, fxp_bits=fxp_bits, seeds=seeds)
            cl.handshake()
            stats = []
            # one result array for every round (checksummed chunk by chunk as it
            # arrives), or a ring of two chunks when only the checksum is kept
            ce = max(1, min(n, chunk_elems()))
            res = np.empty(n, dtype=np.float64) if keep_results else [np.empty(ce, dtype=np.float64)
                                                                       for _ in range(2)]
            after = os.environ.get("SFL_LOOPBACK_CLIENT_RX", "concurrent") == "after"
            for r in range(rounds):
                if after:  # A/B only (round 2's client): read the result once everything is sent
                    st = cl.submit(xs[r], r, weight)
                    cl.result(n, into=res)
                else:
                    st = cl.submit(xs[r], r, weight, result_into=res)
                    cl.result(n)
                st["result_xor"] = cl.last_result_xor
                st["stages"]["client: result recv thread (socket -> numpy, from the start of submit)"] = dict(
                    cl.last_result_recv, calls=1)
                stats.append(st)
            W.recv_header(cl.sock, expect_kind=W.BYE)
            cl.close()
            out_q.put((index, "ok", stats))
        except Exception as e:  # reported to the parent, which fails loudly
            out_q.put((index, "error", repr(e)))

    ts = [threading.Thread(target=run, args=p) for p in parties]
    for t in ts:
        t.start()
    for t in ts:
        t.join()


def run_loopback(names: list[str], n: int, rounds: int = 1, *, seeds: dict | None = None, weights=None,
                 average: bool = False, gpu: int = 0, fxp_bits: int = 18, keep_masked: bool = False,
                 verify_digest: bool = False, timeout: float = 600.0, parties_per_process: int = 1,
                 keep_results: bool = True, gpus: list[int] | None = None, server_gpu: int | None = None):
    """Spawn the client parties (``parties_per_process`` per OS process), run
    ``rounds`` rounds with this process as the server.  Returns (results per
    round, server timings, client stats, received masked vectors).
    ``gpus``: client process g runs on ``gpus[g % len(gpus)]``, the server on
    ``server_gpu`` (default ``gpus[0]``; ``placement``); without it every
    party is on ``gpu``.  ``keep_results=False``: neither the server nor the
    clients keep each round's result (results holds None per round); every
    client checksums what it received either way
    (``stats[i][r]["result_xor"]``)."""
    import multiprocessing as mp

    ctx = mp.get_context("spawn")
    k = max(1, int(parties_per_process))
    n_procs = -(-len(names) // k)
    srv_gpu, proc_gpus = placement(n_procs, list(gpus) if gpus else [gpu], server_gpu)
    srv = LoopbackServer(len(names), gpu=srv_gpu, fxp_bits=fxp_bits)
    q = ctx.Queue()
    procs = []
    specs = []
    for i, p in enumerate(names):
        ps = None if seeds is None else {v: seeds[p][v] for v in names if v != p}
        specs.append((p, i, ps, None if weights is None else weights[i]))
    for g in range(n_procs):
        pr = ctx.Process(target=client_process, args=(specs[g * k:(g + 1) * k], srv.port, n, rounds, proc_gpus[g],
                                                      fxp_bits, q, keep_results))
        pr.start()
        procs.append(pr)
    results, timings, masked = [], [], []
    placed = {"server_gpu": srv_gpu, "client_process_gpus": proc_gpus, "parties_per_process": k}
    try:
        srv.accept(timeout=timeout)
        for r in range(rounds):
            t_start = time.perf_counter()
            out, t = srv.round(n, r, average=average, keep_masked=keep_masked, verify_digest=verify_digest,
                               copy_out=keep_results)
            t["t_start"] = t_start  # successive starts give the steady-state period (copy-out included)
            t["placement"] = placed
            results.append(out if keep_results else None)
            timings.append(t)
            if keep_masked:
                masked.append(srv.last_masked)
    finally:
        srv.close()
    stats = {}
    for _ in names:
        idx, status, payload = q.get(timeout=timeout)
        if status != "ok":
            raise RuntimeError(f"client {idx} failed: {payload}")
        stats[idx] = payload
    for pr in procs:
        pr.join(timeout=60)
    return results, timings, stats, masked
