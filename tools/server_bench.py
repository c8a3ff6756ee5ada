#!/usr/bin/env python3
"""HBM roofline of the server kernels (sfl_amd/csrc/sa_api.hip), not the
headline bench: k_sum_u64 (the wire path's server sum, k masked vectors),
k_decode (scalar divisor: the sum / unweighted average; per-element divisor
vector: per-element weights) and k_sum_f64 (the divisor vector's sum of
weight arrays), each at --elems element positions, timed with HIP events
(median of --reps launches after warm-up), one JSON line per kernel with its
algorithmic bytes and the fraction of the 8 TB/s HBM peak.

Algorithmic bytes per element position (each input read once, the output
written once): k_sum_u64 8(k+1); k_decode 16 (scalar divisor) or 24 (divisor
vector); k_sum_f64 8(k+1).

usage: python tools/server_bench.py [--elems N] [--reps R] [--k 8]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
HBM_PEAK_GBPS = 8000.0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--elems", type=int, default=100_000_000)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--k", type=int, default=8, help="inputs of the u64 / f64 sums")
    args = ap.parse_args()
    import torch

    from sfl_amd import _lib
    from sfl_amd import kernels as K

    _lib.lib()
    dev = torch.device("cuda", 0)
    n, k = args.elems, args.k
    g = torch.Generator(device=dev).manual_seed(5)
    ins = [torch.randint(-2**62, 2**62, (n,), generator=g, device=dev, dtype=torch.int64) for _ in range(k)]
    su = torch.empty(n, dtype=torch.int64, device=dev)
    dec = torch.empty(n, dtype=torch.float64, device=dev)
    dv = torch.rand(n, generator=g, device=dev, dtype=torch.float64) + 1.0
    fins = [torch.rand(n, generator=g, device=dev, dtype=torch.float64) for _ in range(k)]
    fo = torch.empty(n, dtype=torch.float64, device=dev)
    cases = [
        ("k_sum_u64", f"sa_sum_u64 of {k} masked vectors", 8 * (k + 1), lambda: K.sum_u64(ins, su)),
        ("k_decode<false>", "sa_decode, scalar divisor", 16, lambda: K.decode(ins[0], dec, divisor=3.0)),
        ("k_decode<true>", "sa_decode, per-element divisor vector", 24,
         lambda: K.decode(ins[0], dec, divisor_vec=dv)),
        ("k_sum_f64", f"sa_sum_f64 of {k} weight arrays", 8 * (k + 1), lambda: K.sum_f64(fins, fo)),
    ]
    for name, what, bpe, fn in cases:
        for _ in range(5):
            fn()
        times = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            times.append(e0.elapsed_time(e1))
        times.sort()
        ms = times[len(times) // 2]
        gbps = bpe * n / (ms / 1e3) / 1e9
        print(json.dumps({"kernel": name, "what": what, "elems": n, "algorithmic_bytes": bpe * n,
                          "ms_median": ms, "ms_min": times[0], "GBps": gbps, "hbm_frac": gbps / HBM_PEAK_GBPS}),
              flush=True)


if __name__ == "__main__":
    main()
