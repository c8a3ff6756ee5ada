#!/usr/bin/env python3
"""BASELINE config 1 through the plugin surface: 2 parties, a 1M-element
numpy vector each (float64 like the notebook KAT, and float32 like the FL
payloads), ``SecureAggregator.sum`` / ``.average`` host array in -> host array
out (H2D, fused quantize + mask + sum, decode, D2H all inside the call), timed
beside the numpy restatement (oracle/secagg.py, the reference's CPU path, one
core) on the same inputs.  The first call of each kind is checked against the
oracle (decoded result bit-exact); the timed calls advance the streams like
consecutive rounds.

usage: python tools/config1_bench.py [--elems 1000000] [--reps 50]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--elems", type=int, default=1_000_000)
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--cpu-reps", type=int, default=5)
    args = ap.parse_args()
    import numpy as np
    import torch

    from oracle import secagg as o
    from sfl_amd.device import PYU, PYUObject
    from sfl_amd.security.aggregation import SecureAggregator

    names = ["alice", "bob"]
    seeds = o.seeds_for(names)
    pyus = [PYU(n, 0) for n in names]
    server = PYU("carol", 0)
    rng = np.random.default_rng(20260116)
    out = {"config": "BASELINE config 1: 2 parties x %d-element numpy vector, fxp 18, ring 2^64" % args.elems,
           "path": "SecureAggregator.sum/average on host numpy arrays (H2D + fused launch + decode + D2H per call)",
           "cases": []}
    for dt in (np.float64, np.float32):
        xs = [rng.random(args.elems).astype(dt) for _ in names]  # np.random.rand-style, as the KAT
        for kind in ("sum", "average"):
            agg = SecureAggregator(server, pyus, seeds={(a, b): seeds[a][b] for a in names for b in names if a < b})
            objs = [PYUObject(p, x) for p, x in zip(pyus, xs)]
            fn = getattr(agg, kind)
            first = fn(objs, axis=0).data
            torch.cuda.synchronize()
            ref = (o.secure_sum(xs, names, seeds=seeds)[0] if kind == "sum"
                   else o.secure_average(xs, names, seeds=seeds)[0])
            exact = bool(np.array_equal(first, ref))
            tol = float(np.max(np.abs(first - (xs[0].astype(np.float64) + xs[1]) / (1 if kind == "sum" else 2))))
            for _ in range(20):  # clocks ramp after idle
                fn(objs, axis=0)
            ts = []
            for _ in range(args.reps):
                t0 = time.perf_counter()
                fn(objs, axis=0)
                ts.append(time.perf_counter() - t0)
            cpu = []
            for i in range(args.cpu_reps):
                t0 = time.perf_counter()
                if kind == "sum":
                    o.secure_sum(xs, names, seeds=seeds, offset=i * args.elems)
                else:
                    o.secure_average(xs, names, seeds=seeds, offset=i * args.elems)
                cpu.append(time.perf_counter() - t0)
            g, c = float(np.median(ts)), float(np.median(cpu))
            out["cases"].append({
                "dtype": np.dtype(dt).name, "op": kind, "bit_exact_vs_oracle": exact,
                "max_abs_err_vs_float_sum": tol,
                "hip_ms_median": g * 1e3, "hip_grad_elems_per_s": 2 * args.elems / g,
                "cpu_numpy_ms_median": c * 1e3, "cpu_grad_elems_per_s": 2 * args.elems / c,
                "speedup": c / g})
    print(json.dumps(out))


if __name__ == "__main__":
    main()
