#!/usr/bin/env python3
"""Host <-> device copy paths for the drop-in's large payloads (one party's
100M-float gradient in, its 100M uint64 masked vector out), measured on the
GPU box: what floor the per-party functions (party.mask_payload,
party.sum_decode) can reach from pageable numpy arrays.

Prints one JSON line per measurement (GB/s of payload bytes, medians):
  pinned_h2d / pinned_d2h / pinned_bidir   page-locked staging, one / both directions
  pageable_h2d / pageable_d2h               torch's own pageable copies (the round-5 path)
  register_{in,out}                         hipHostRegister of a caller array (+ unregister)
  memcpy_threads_<k>                        numpy copy pageable -> pinned on k threads
  fresh_out_touch                           np.empty(800 MB) first touch (page faults)
usage: python tools/pcie_paths.py [--mb 400]
"""
import argparse
import ctypes
import json
import os
import statistics
import sys
import threading
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def med(fn, reps=5):
    ts = []
    for _ in range(reps):
        t0 = time.perf_counter()
        fn()
        ts.append(time.perf_counter() - t0)
    return statistics.median(ts)


def emit(name, nbytes, s, **kw):
    print(json.dumps({"path": name, "bytes": nbytes, "ms": s * 1e3, "GBps": nbytes / s / 1e9, **kw}), flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--mb", type=int, default=400, help="input MB (the output is twice that)")
    a = ap.parse_args()
    import torch

    dev = torch.device("cuda", 0)
    nin = a.mb << 20
    nout = 2 * nin
    x = np.random.default_rng(1).integers(0, 255, nin, dtype=np.uint8)
    out = np.empty(nout, dtype=np.uint8)
    out[:] = 1
    d_in = torch.empty(nin, dtype=torch.uint8, device=dev)
    d_out = torch.empty(nout, dtype=torch.uint8, device=dev)
    p_in = torch.empty(nin, dtype=torch.uint8, pin_memory=True)
    p_out = torch.empty(nout, dtype=torch.uint8, pin_memory=True)
    s1, s2 = torch.cuda.Stream(dev), torch.cuda.Stream(dev)

    def h2d():
        d_in.copy_(p_in, non_blocking=True)
        torch.cuda.synchronize()

    def d2h():
        p_out.copy_(d_out, non_blocking=True)
        torch.cuda.synchronize()

    def bidir():
        with torch.cuda.stream(s1):
            d_in.copy_(p_in, non_blocking=True)
        with torch.cuda.stream(s2):
            p_out.copy_(d_out, non_blocking=True)
        torch.cuda.synchronize()

    h2d(), d2h()
    emit("pinned_h2d", nin, med(h2d))
    emit("pinned_d2h", nout, med(d2h))
    emit("pinned_bidir", nin + nout, med(bidir), note="H2D of the input and D2H of the output on two streams")

    tx = torch.from_numpy(x)
    tout = torch.from_numpy(out)

    def pg_h2d():
        d_in.copy_(tx)
        torch.cuda.synchronize()

    def pg_d2h():
        tout.copy_(d_out)
        torch.cuda.synchronize()

    emit("pageable_h2d", nin, med(pg_h2d))
    emit("pageable_d2h", nout, med(pg_d2h), note="into an already-touched numpy array")

    def fresh():
        o = np.empty(nout, dtype=np.uint8)
        o[::4096] = 0
        return o

    emit("fresh_out_touch", nout, med(fresh, 3), note="np.empty + one write per 4 KiB page")

    hip = ctypes.CDLL("libamdhip64.so")

    def reg(arr):
        def f():
            p = ctypes.c_void_p(arr.ctypes.data)
            rc = hip.hipHostRegister(p, ctypes.c_size_t(arr.nbytes), ctypes.c_uint(0))
            assert rc == 0, rc
            rc = hip.hipHostUnregister(p)
            assert rc == 0, rc
        return f

    emit("register_in", nin, med(reg(x), 3), note="hipHostRegister + hipHostUnregister of the touched input")
    emit("register_out", nout, med(reg(out), 3), note="same, the touched output")
    # registered input: H2D straight from the caller's pages
    p = ctypes.c_void_p(x.ctypes.data)
    assert hip.hipHostRegister(p, ctypes.c_size_t(nin), ctypes.c_uint(0)) == 0
    emit("registered_h2d", nin, med(pg_h2d))
    hip.hipHostUnregister(p)

    pv_in = p_in.numpy()
    for k in (1, 2, 4, 8, 16):
        def cp(k=k):
            step = -(-nin // k)
            ths = [threading.Thread(target=np.copyto, args=(pv_in[i:i + step], x[i:i + step]))
                   for i in range(0, nin, step)]
            for t in ths:
                t.start()
            for t in ths:
                t.join()
        emit(f"memcpy_threads_{k}", nin, med(cp), note="pageable numpy -> pinned, k threads")


if __name__ == "__main__":
    main()
