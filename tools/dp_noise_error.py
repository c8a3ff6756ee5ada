#!/usr/bin/env python3
"""Error of the device's Box-Muller noise (sa_philox.h) against the numpy
restatement in oracle/dp.py (accurate libm), over --n normals: max absolute
error, max error relative to max(|z|, 1), and the moments of both."""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--n", type=int, default=4_000_000)
    args = ap.parse_args()
    import numpy as np
    import torch

    from oracle import dp as D
    from sfl_amd import _lib as L
    from sfl_amd import kernels as K

    dev = torch.device("cuda", 0)
    key, n = 0x1234_5678_9ABC_DEF0, args.n
    s = torch.zeros(1, dtype=torch.float64, device=dev)
    part = torch.empty(L.SA_DP_PARTIALS, dtype=torch.float64, device=dev)
    K.sumsq_f32(torch.ones(4, device=dev), s, part)
    dp = K.make_dp(s, l2_norm_clip=1e9, noise_std=1.0, num_updates=1.0, key=key, counter0=0)
    z = K.dp_perturb(torch.zeros(n, device=dev), torch.empty(n, device=dev), dp).cpu().numpy().astype(np.float64)
    ref = D.gauss(key, 0, n).astype(np.float64)
    err = np.abs(z - ref)
    print(json.dumps({"n": n, "max_abs_err": float(err.max()), "max_err_rel_to_max_abs_z_1":
                      float((err / np.maximum(np.abs(ref), 1.0)).max()), "mean": [float(z.mean()), float(ref.mean())],
                      "std": [float(z.std()), float(ref.std())], "max_abs": [float(np.abs(z).max()), float(np.abs(ref).max())]}))


if __name__ == "__main__":
    main()
