#!/usr/bin/env python3
"""Fresh host result buffers on the GPU box: how fast 800 MB of fresh
memory can be faulted in (np.empty vs an anonymous mmap; 1 or 8 threads;
8 or 64 tasks), what hipHostRegister of it costs (touched / untouched,
whole / 8 chunks, with the GPU idle), and the D2H rate into it (registered
vs pageable).  One JSON line per measurement.  Feeds sfl_amd/hostpipe.py's
choice of how the pipelined drop-in writes its results."""
import ctypes
import json
import mmap
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

PAGE = 4096
NB = 800 << 20
hip = ctypes.CDLL("libamdhip64.so")
pool = ThreadPoolExecutor(8)


def emit(what, ms, **kw):
    print(json.dumps({"what": what, "ms": round(ms, 3), "GBps": round(NB / ms / 1e6, 1), **kw}), flush=True)


def alloc(kind):
    if kind == "np":
        return np.empty(NB, dtype=np.uint8), None
    mm = mmap.mmap(-1, NB, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
    return np.frombuffer(mm, dtype=np.uint8), mm


def touch(b, tasks, threads):
    step = -(-NB // tasks) // PAGE * PAGE

    def t(lo):
        b[lo:lo + step:PAGE] = 0

    if threads == 1:
        for lo in range(0, NB, step):
            t(lo)
    else:
        list(pool.map(t, range(0, NB, step)))


def reg(b, parts=1):
    step = NB // parts
    t0 = time.perf_counter()
    for lo in range(0, NB, step):
        assert hip.hipHostRegister(ctypes.c_void_p(b.ctypes.data + lo), ctypes.c_size_t(step), ctypes.c_uint(0)) == 0
    t1 = time.perf_counter()
    for lo in range(0, NB, step):
        hip.hipHostUnregister(ctypes.c_void_p(b.ctypes.data + lo))
    return 1e3 * (t1 - t0), 1e3 * (time.perf_counter() - t1)


def main():
    import torch

    dev = torch.device("cuda", 0)
    src = torch.empty(NB, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    for kind in ("np", "mmap"):
        for threads, tasks in ((1, 1), (8, 8), (8, 64)):
            b, mm = alloc(kind)
            t0 = time.perf_counter()
            touch(b, tasks, threads)
            emit(f"touch {kind} threads={threads} tasks={tasks}", 1e3 * (time.perf_counter() - t0))
            del b, mm
        for touched in (True, False):
            for parts in (1, 8):
                b, mm = alloc(kind)
                if touched:
                    touch(b, 8, 8)
                r, u = reg(b, parts)
                emit(f"register {kind} touched={touched} parts={parts}", r, unregister_ms=round(u, 3))
                del b, mm
        for mode in ("registered", "pageable"):
            b, mm = alloc(kind)
            touch(b, 8, 8)
            if mode == "registered":
                assert hip.hipHostRegister(ctypes.c_void_p(b.ctypes.data), ctypes.c_size_t(NB), ctypes.c_uint(0)) == 0
            dst = torch.from_numpy(b)
            ts = []
            for _ in range(4):
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                dst.copy_(src, non_blocking=True)
                torch.cuda.synchronize()
                ts.append(1e3 * (time.perf_counter() - t0))
            emit(f"d2h {kind} {mode}", min(ts[1:]), first_ms=round(ts[0], 3))
            if mode == "registered":
                hip.hipHostUnregister(ctypes.c_void_p(b.ctypes.data))
            del dst, b, mm
        # fresh, untouched, pageable D2H: the runtime faults the pages itself
        b, mm = alloc(kind)
        dst = torch.from_numpy(b)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        dst.copy_(src, non_blocking=True)
        torch.cuda.synchronize()
        emit(f"d2h {kind} pageable untouched", 1e3 * (time.perf_counter() - t0))
        del dst, b, mm


if __name__ == "__main__":
    main()
