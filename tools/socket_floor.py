#!/usr/bin/env python3
"""The loopback transport floor of one secure-aggregation round, without a GPU.

What a round of sfl_amd/loopback.py must move through TCP on 127.0.0.1 no
matter how fast the GPU is: every client sends its masked uint64 vector (8n
bytes) to the server, the server sends the float64 result (8n bytes) back to
every client.  Here C client processes and a server with one receive and one
send thread per client do exactly that with preallocated buffers and nothing
else (no H2D / D2H, no kernels, no staging copies): the time is the cost of
the socket copies alone -- per direction one copy into the kernel on send
and one out of it on receive.

``--sendfile``: the payloads leave from a memfd through os.sendfile (page
references handed to the socket, no copy on the send side), so each byte is
copied once, on receive.  ``--overlap``: the result goes back while the
masked vectors are still arriving (the pipelined server's schedule: its
broadcast of chunk j overlaps the reception of later chunks), so both
directions run at once.

usage: python tools/socket_floor.py [--clients 8] [--elems 100000000] [--rounds 4] [--sendfile]
"""
import argparse
import json
import mmap
import multiprocessing as mp
import os
import socket
import sys
import threading
import time

import numpy as np

CHUNK = 64 << 20  # the loopback runtime's staging chunk (8M u64)


def _send(sock, buf: memoryview, fd: int | None, nbytes: int):
    if fd is not None and sock.gettimeout() is not None:  # socket.sendfile: poll + os.sendfile
        f = open(fd, "rb", buffering=0, closefd=False)
        off = 0
        while off < nbytes:
            k = min(CHUNK, nbytes - off)
            assert sock.sendfile(f, off, k) == k
            off += k
        f.close()
        return
    if fd is None:
        off = 0
        while off < nbytes:
            k = min(CHUNK, nbytes - off)
            sock.sendall(buf[off:off + k])
            off += k
    else:
        off = 0
        while off < nbytes:
            off += os.sendfile(sock.fileno(), fd, off, nbytes - off)


def _recv(sock, buf: memoryview, nbytes: int):
    got = 0
    while got < nbytes:
        k = sock.recv_into(buf[got:], min(CHUNK, nbytes - got))
        if k == 0:
            raise ConnectionError("closed")
        got += k


def _memfd(nbytes: int):
    fd = os.memfd_create("sfl_socket_floor")
    os.ftruncate(fd, nbytes)
    mm = mmap.mmap(fd, nbytes)
    np.frombuffer(mm, dtype=np.uint8)[:] = 7  # fault the pages in
    return fd, mm


def client(port: int, nbytes: int, rounds: int, sendfile: bool, overlap: bool, timeout, q, client_overlap=True):
    """One client: sends its masked vector, receives the result (concurrently with --overlap)."""
    try:
        s = socket.create_connection(("127.0.0.1", port), timeout=timeout)
        s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        if sendfile:
            fd, mm = _memfd(nbytes)
            out = memoryview(mm)
        else:
            fd, out = None, memoryview(np.full(nbytes, 7, dtype=np.uint8))
        res = memoryview(np.empty(nbytes, dtype=np.uint8))
        for _ in range(rounds):
            if overlap and client_overlap:
                t = threading.Thread(target=_recv, args=(s, res, nbytes))
                t.start()
                _send(s, out, fd, nbytes)
                t.join()
            else:
                _send(s, out, fd, nbytes)
                _recv(s, res, nbytes)
        s.close()
        q.put("ok")
    except Exception as e:  # noqa: BLE001
        q.put(repr(e))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--elems", type=int, default=100_000_000)
    ap.add_argument("--rounds", type=int, default=4)
    ap.add_argument("--sendfile", action="store_true", help="both directions")
    ap.add_argument("--sendfile-side", choices=("both", "clients", "server"), default="both",
                    help="with --sendfile: which senders use it")
    ap.add_argument("--overlap", action="store_true")
    ap.add_argument("--client-sequential", action="store_true",
                    help="with --overlap: clients read the result only after sending everything (the loopback "
                         "runtime's client), while the server already sends")
    ap.add_argument("--timeout", type=float, default=None,
                    help="sockets with a timeout (non-blocking descriptors; sendfile through socket.sendfile)")
    args = ap.parse_args()
    C, nbytes = args.clients, 8 * args.elems
    srv = socket.create_server(("127.0.0.1", 0))
    port = srv.getsockname()[1]
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    procs = [ctx.Process(target=client, args=(port, nbytes, args.rounds, args.sendfile and args.sendfile_side != "server",
                                                   args.overlap, args.timeout, q,
                                                   not args.client_sequential)) for _ in range(C)]
    for p in procs:
        p.start()
    conns = []
    for _ in range(C):
        c, _ = srv.accept()
        c.settimeout(args.timeout)
        c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        conns.append(c)
    rx = [memoryview(np.empty(nbytes, dtype=np.uint8)) for _ in range(C)]
    if args.sendfile and args.sendfile_side != "clients":
        fd, mm = _memfd(nbytes)
        res = memoryview(mm)
    else:
        fd, res = None, memoryview(np.full(nbytes, 3, dtype=np.uint8))
    times = []
    for _ in range(args.rounds):
        t0 = time.perf_counter()
        rt = [threading.Thread(target=_recv, args=(conns[i], rx[i], nbytes)) for i in range(C)]
        st = [threading.Thread(target=_send, args=(conns[i], res, fd, nbytes)) for i in range(C)]
        for t in rt:
            t.start()
        if args.overlap:
            for t in st:
                t.start()
        for t in rt:
            t.join()
        t1 = time.perf_counter()
        if not args.overlap:
            for t in st:
                t.start()
        for t in st:
            t.join()
        times.append((t1 - t0, time.perf_counter() - t1))
    for p in procs:
        p.join(timeout=120)
    errs = [q.get(timeout=10) for _ in procs]
    if any(e != "ok" for e in errs):
        raise SystemExit(f"client failed: {errs}")
    steady = times[1:] or times
    rx_s = float(np.median([a for a, _ in steady]))
    tx_s = float(np.median([b for _, b in steady]))
    round_s = float(np.median([a + b for a, b in steady]))
    print(json.dumps({"what": "loopback transport floor (no GPU): C masked u64 vectors in, the float64 result "
                              "back to every client", "send": f"os.sendfile from a memfd ({args.sendfile_side})" if args.sendfile
                      else "sendall from user memory", "client_sequential": args.client_sequential, "overlap": args.overlap, "socket_timeout": args.timeout, "clients": C, "elems": args.elems, "rounds": args.rounds,
                      "gather_s": rx_s, "after_gather_s": tx_s, "round_s": round_s,
                      "wire_GBps": 2 * C * nbytes / round_s / 1e9,
                      "grad_elems_per_s": C * args.elems / round_s, "cpus": os.cpu_count(),
                      "cpus_usable": len(os.sched_getaffinity(0))}), flush=True)


if __name__ == "__main__":
    sys.exit(main())
