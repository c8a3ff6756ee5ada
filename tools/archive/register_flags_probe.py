#!/usr/bin/env python3
"""hipHostRegister cost by flag on the GPU box: 1 GB touched numpy arrays
registered whole and in 64 MB pieces with hipHostRegisterDefault (0),
Mapped (2) and ReadOnly (8), and the H2D rate out of each registration.
One JSON line per case.  Feeds hostpipe.Pinned's flag choice."""
import ctypes
import json
import time

import numpy as np
import torch

hip = ctypes.CDLL("libamdhip64.so")
NB = 1 << 30
PIECE = 64 << 20


def main():
    dev = torch.device("cuda", 0)
    d = torch.empty(NB, dtype=torch.uint8, device=dev)
    torch.cuda.synchronize()
    for flags in (0, 2, 8):
        for piece in (NB, PIECE):
            ts, tu, rate = [], [], []
            for _ in range(3):
                a = np.ones(NB, np.uint8)
                t0 = time.perf_counter()
                ok = True
                for lo in range(0, NB, piece):
                    rc = hip.hipHostRegister(ctypes.c_void_p(a.ctypes.data + lo), ctypes.c_size_t(piece),
                                             ctypes.c_uint(flags))
                    if rc:
                        hip.hipGetLastError()
                        ok = False
                        break
                ts.append(1e3 * (time.perf_counter() - t0))
                if ok:
                    torch.cuda.synchronize()
                    t0 = time.perf_counter()
                    for lo in range(0, NB, piece):
                        d[lo:lo + piece].copy_(torch.from_numpy(a[lo:lo + piece]), non_blocking=True)
                    torch.cuda.synchronize()
                    rate.append(NB / (time.perf_counter() - t0) / 1e9)
                    t0 = time.perf_counter()
                    for lo in range(0, NB, piece):
                        hip.hipHostUnregister(ctypes.c_void_p(a.ctypes.data + lo))
                    tu.append(1e3 * (time.perf_counter() - t0))
                del a
            print(json.dumps({"flags": flags, "piece_MB": piece >> 20, "ok": ok,
                              "register_ms": [round(t, 2) for t in ts], "unregister_ms": [round(t, 2) for t in tu],
                              "h2d_GBps": [round(r, 1) for r in rate]}), flush=True)


if __name__ == "__main__":
    main()
