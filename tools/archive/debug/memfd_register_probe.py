#!/usr/bin/env python3
"""Probe: can a memfd-backed host buffer be HIP-registered (hipHostRegister)
so a D2H copy lands in it directly and os.sendfile then ships its pages
without a send-side copy?  Checks registration, torch's view of it as
pinned, a non-blocking D2H into it (bit-exact), and the D2H rate against a
hipHostMalloc'ed (torch pin_memory) buffer."""
import ctypes as C
import json
import mmap
import os
import time

import numpy as np
import torch


def main():
    n = 100_000_000
    nbytes = 8 * n
    hip = C.CDLL("libamdhip64.so")
    fd = os.memfd_create("probe")
    os.ftruncate(fd, nbytes)
    mm = mmap.mmap(fd, nbytes)
    a = np.frombuffer(mm, dtype=np.uint64)
    a[:] = 0  # fault in
    ptr = a.ctypes.data
    t0 = time.perf_counter()
    rc = hip.hipHostRegister(C.c_void_p(ptr), C.c_size_t(nbytes), C.c_uint(0))
    t_reg = time.perf_counter() - t0
    t = torch.from_numpy(a.view(np.int64))
    dev = torch.device("cuda", 0)
    d = torch.randint(-2**62, 2**62, (n,), device=dev, dtype=torch.int64)
    s = torch.cuda.Stream(dev)
    res = {"hipHostRegister_rc": rc, "register_s": t_reg, "torch_is_pinned": bool(t.is_pinned())}
    for rep in range(3):
        with torch.cuda.stream(s):
            t0 = time.perf_counter()
            t.copy_(d, non_blocking=True)
            t_enq = time.perf_counter() - t0
            s.synchronize()
            t_all = time.perf_counter() - t0
    res.update({"d2h_enqueue_s": t_enq, "d2h_s": t_all, "d2h_GBps": nbytes / t_all / 1e9,
                "bit_exact": bool(torch.equal(t, d.cpu()))})
    p = torch.empty(n, dtype=torch.int64).pin_memory()
    with torch.cuda.stream(s):
        for rep in range(3):
            t0 = time.perf_counter()
            p.copy_(d, non_blocking=True)
            s.synchronize()
            t_p = time.perf_counter() - t0
    res["pinned_d2h_GBps"] = nbytes / t_p / 1e9
    # H2D from it as well
    with torch.cuda.stream(s):
        for rep in range(3):
            t0 = time.perf_counter()
            d.copy_(t, non_blocking=True)
            s.synchronize()
            t_h = time.perf_counter() - t0
    res["h2d_GBps"] = nbytes / t_h / 1e9
    res["unregister_rc"] = hip.hipHostUnregister(C.c_void_p(ptr))
    print(json.dumps(res))


if __name__ == "__main__":
    main()
