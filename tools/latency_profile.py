#!/usr/bin/env python3
"""Where a small SecureAggregator.sum call spends its time: cProfile over
many calls of 2 parties x n host elements (float32 and float64), top
functions by own time.  A measurement tool, not the product.

usage: python tools/latency_profile.py [--elems 99] [--calls 2000]
"""
import argparse
import cProfile
import io
import os
import pstats
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--elems", type=int, default=99)
    ap.add_argument("--calls", type=int, default=2000)
    ap.add_argument("--top", type=int, default=30)
    args = ap.parse_args()
    import numpy as np
    import torch

    from sfl_amd.device import PYU, PYUObject
    from sfl_amd.security.aggregation import SecureAggregator

    names = ["alice", "bob"]
    pyus = [PYU(n, 0) for n in names]
    server = PYU("carol", 0)
    rng = np.random.default_rng(1)
    from sfl_amd.compat import secretflow as hip_compat

    cases = [(dt, SecureAggregator) for dt in (np.float32, np.float64, np.int64)]
    cases.append((np.float32, hip_compat.SecureAggregator))  # the per-party drop-in, in-process devices
    for dt, cls in cases:
        xs = [(rng.random(args.elems) * 1000).astype(dt) for _ in names]
        agg = cls(server, pyus)
        objs = [PYUObject(p, x) for p, x in zip(pyus, xs)]
        for _ in range(200):
            agg.sum(objs, axis=0)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.calls):
            agg.sum(objs, axis=0)
        per = (time.perf_counter() - t0) / args.calls
        pr = cProfile.Profile()
        pr.enable()
        for _ in range(args.calls):
            agg.sum(objs, axis=0)
        pr.disable()
        s = io.StringIO()
        pstats.Stats(pr, stream=s).sort_stats("tottime").print_stats(args.top)
        print(f"==== {np.dtype(dt).name} {cls.__module__}: {per * 1e6:.1f} us per call (unprofiled)")
        print(s.getvalue())


if __name__ == "__main__":
    main()
