#!/usr/bin/env python3
"""Rooflines of the fused DP pre-step (sfl_amd/csrc/sa_dp.hip)
against the masking it rides on, one client of --elems float32 elements:

* k_sumsq_partial + k_sumsq_final: the clipping norm, sum(x^2) in float64
  (4 B read per element: HBM-bound);
* k_dp_perturb standalone: x * min(1, clip/||x||) + Philox-Box-Muller noise
  (4 B read + 4 B written per element);
* sa_mask of one client with --streams pair streams, without DP (the lean
  kernel) and with the perturbation fused in (sa_mask_dp: the noise is drawn
  inside the masking kernel on the loaded tile, no extra HBM pass), and the
  unfused alternative (perturb, then mask) for comparison.

Median of --reps launches per pass (HIP events), the cases interleaved over
--passes after a clock warm-up; one JSON line per case (median of the passes).
usage: python tools/dp_bench.py [--elems 100000000] [--streams 7] [--reps 20] [--passes 3]
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
    ap.add_argument("--streams", type=int, default=7)
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--passes", type=int, default=3)
    ap.add_argument("--warmup", type=int, default=30, help="lean masking launches before the first case")
    args = ap.parse_args()
    import torch

    from bench import pair_seed
    from sfl_amd import _lib as L
    from sfl_amd import kernels as K

    L.lib()
    dev = torch.device("cuda", 0)
    n = args.elems
    g = torch.Generator(device=dev).manual_seed(3)
    x = torch.randn(n, generator=g, device=dev, dtype=torch.float32) * 1e-2
    xp = torch.empty_like(x)
    out = torch.empty(n, dtype=torch.int64, device=dev)
    ss = torch.zeros(1, dtype=torch.float64, device=dev)
    partials = torch.zeros(L.SA_DP_PARTIALS, dtype=torch.float64, device=dev)
    K.sumsq_f32(x, ss, partials)
    dp = K.make_dp(ss, l2_norm_clip=1.0, noise_std=0.5, num_updates=8.0, key=1234)
    streams = [(L.pcg64_from_seed(pair_seed(0, v + 1)), 1 if v % 2 else -1, v) for v in range(args.streams)]

    def time(fn):
        for _ in range(min(5, args.reps)):
            fn()
        ts = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            fn()
            e1.record()
            e1.synchronize()
            ts.append(e0.elapsed_time(e1))
        ts.sort()
        return ts[len(ts) // 2]

    cases = [
        ("k_sumsq (clipping norm)", 4, lambda: K.sumsq_f32(x, ss, partials)),
        ("k_dp_perturb (standalone)", 8, lambda: K.dp_perturb(x, xp, dp)),
        (f"sa_mask, {args.streams} streams, no DP (lean kernel)", 12, lambda: K.mask(x, out, streams)),
        (f"sa_mask_dp, {args.streams} streams (perturbation fused)", 12, lambda: K.mask_dp(x, out, streams, dp)),
        (f"dp_perturb then sa_mask, {args.streams} streams (unfused)", 20,
         lambda: (K.dp_perturb(x, xp, dp), K.mask(xp, out, streams))),
    ]
    # warm the clocks, then interleave the cases over passes (the first
    # launches after idle run at lower clocks)
    for _ in range(args.warmup):
        K.mask(x, out, streams)
    res = {name: [] for name, _, _ in cases}
    for _ in range(args.passes):
        for name, _, fn in cases:
            res[name].append(time(fn))
    for name, bpe, _ in cases:
        v = sorted(res[name])
        ms = v[len(v) // 2]
        gbps = bpe * n / (ms / 1e3) / 1e9
        print(json.dumps({"case": name, "elems": n, "algorithmic_bytes": bpe * n, "ms_median": ms,
                          "ms_passes": v, "GBps": gbps, "hbm_frac": gbps / HBM_PEAK_GBPS}), flush=True)


if __name__ == "__main__":
    main()
