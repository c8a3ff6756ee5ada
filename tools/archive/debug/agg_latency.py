"""Latency of one SecureAggregator.average call at the FL-round size (config
4: 8 parties, MlpNet 4-50-50-3 = 2,953 float32 parameters in 6 host arrays,
integer sample-count weights), with a cProfile breakdown of where the host
time goes.  usage: python tools/debug/agg_latency.py [--reps 200]"""
import argparse
import cProfile
import os
import pstats
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
import numpy as np  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=200)
    ap.add_argument("--torch-payload", action="store_true", help="payload as cuda tensors instead of numpy")
    args = ap.parse_args()
    import torch

    from oracle import secagg as o
    from sfl_amd.device import PYU, PYUObject, reveal
    from sfl_amd.security.aggregation import SecureAggregator

    names = [f"party{c}" for c in range(8)]
    seeds = o.seeds_for(names)
    pair = {(a, b): seeds[a][b] for a in names for b in names if a != b}
    pyus = [PYU(n, 0) for n in names]
    agg = SecureAggregator(PYU("server", 0), pyus, seeds=pair)
    shapes = [(4, 50), (50,), (50, 50), (50,), (50, 3), (3,)]
    rng = np.random.default_rng(0)
    payloads = [[rng.standard_normal(s).astype(np.float32) * 0.1 for s in shapes] for _ in names]
    if args.torch_payload:
        payloads = [[torch.from_numpy(a).cuda() for a in p] for p in payloads]
    nums = [960] * 8

    def call():
        r = agg.average([PYUObject(d, p) for d, p in zip(pyus, payloads)], axis=0, weights=nums)
        out = reveal(r)
        if args.torch_payload:
            torch.cuda.synchronize()
        return out

    for _ in range(20):
        call()
    ts = []
    for _ in range(args.reps):
        t0 = time.perf_counter()
        call()
        ts.append(time.perf_counter() - t0)
    print(f"average(): median {1e3 * np.median(ts):.3f} ms, min {1e3 * min(ts):.3f} ms over {args.reps}")
    pr = cProfile.Profile()
    pr.enable()
    for _ in range(50):
        call()
    pr.disable()
    pstats.Stats(pr).sort_stats("tottime").print_stats(25)


if __name__ == "__main__":
    main()
