#!/usr/bin/env python3
"""hipHostRegister of 8 x 1 GB touched arrays from 1, 2, 4 and 8 threads at
once (one array per task): does registration scale across threads?  Fresh
arrays every trial, and the same arrays registered again after an
unregister (the runtime may keep their mapping).  One JSON line per case
(wall ms, median of 3).  Feeds hostpipe.Pinned."""
import ctypes
import json
import statistics
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import torch

hip = ctypes.CDLL("libamdhip64.so")
NB, K = 1 << 30, 8


def reg(a):
    assert hip.hipHostRegister(ctypes.c_void_p(a.ctypes.data), ctypes.c_size_t(a.nbytes), ctypes.c_uint(0)) == 0


def fresh():
    return [np.ones(NB, np.uint8) for _ in range(K)]


def unreg(arrs):
    for a in arrs:
        hip.hipHostUnregister(ctypes.c_void_p(a.ctypes.data))


def main():
    torch.empty(1, device="cuda:0")
    torch.cuda.synchronize()
    warm = fresh()
    reg(warm[0])  # the process's first registration maps the runtime's state
    unreg(warm[:1])
    del warm
    for threads in (1, 2, 4, 8):
        ts, again = [], []
        for _ in range(3):
            arrs = fresh()
            with ThreadPoolExecutor(threads) as ex:
                t0 = time.perf_counter()
                list(ex.map(reg, arrs))
                ts.append(1e3 * (time.perf_counter() - t0))
                unreg(arrs)
                t0 = time.perf_counter()
                list(ex.map(reg, arrs))
                again.append(1e3 * (time.perf_counter() - t0))
            unreg(arrs)
            del arrs
        print(json.dumps({"threads": threads, "GB": K, "fresh_register_ms": round(statistics.median(ts), 2),
                          "fresh_all_ms": [round(t, 2) for t in ts],
                          "reregister_ms": round(statistics.median(again), 2)}), flush=True)


if __name__ == "__main__":
    main()
