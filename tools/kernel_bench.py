#!/usr/bin/env python3
"""Kernel-level timing of the masking kernels for tuning (not the headline
bench).  Times sa_fused_clients for the per-rank shapes of C clients split
over W GPUs (rank 0's share, no RCCL) and the single-client sa_mask, with
hipEvents, interleaving configurations over several rounds in one process.

usage: python tools/kernel_bench.py [--elems N] [--rounds R] [--shapes 8:1,8:2,8:4,8:8]
Set SFL_SA_LIB to time a tuning variant of libsfl_sa.so.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# timing tool: may load a tuning variant (SFL_SA_LIB) that the product loader refuses
os.environ.setdefault("SFL_SA_ALLOW_TUNING_BUILD", "1")
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--elems", type=int, default=100_000_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--shapes", default="8:1,8:2,8:4,8:8", help="C:W pairs")
    ap.add_argument("--calib", type=int, default=0,
                    help="also launch sa_sum_u64 over this many u64 inputs (known bytes, for PMC calibration)")
    args = ap.parse_args()
    import torch

    from bench import pair_seed
    from sfl_amd import _lib
    from sfl_amd import kernels as K
    from sfl_amd.parallel_sum import plan_generators, plan_rank

    _lib.lib()
    dev = torch.device("cuda", 0)
    N = args.elems
    shapes = [tuple(int(v) for v in s.split(":")) for s in args.shapes.split(",")]
    cases = []
    for C, W in shapes:
        names = [f"client{c}" for c in range(C)]
        plan = plan_rank(names, W, 0)
        xs = [torch.randn(N, device=dev) * 1e-2 for _ in plan.clients]
        pg, ps, cross = plan_generators(plan, pair_seed)
        s = torch.empty(N, dtype=torch.int64, device=dev)
        cases.append(dict(C=C, W=W, L=len(plan.clients), plan=plan, xs=xs, pg=pg, ps=ps, cross=cross, s=s,
                          times=[]))
    for _ in range(args.rounds):
        for cs in cases:
            def run():
                K.fused_clients(cs["xs"], [1.0] * cs["L"], cs["pg"], cs["ps"], cs["cross"], cs["plan"].n_cross,
                                cs["s"])
            run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            cs["times"].append(e0.elapsed_time(e1) / args.reps)
    if args.calib:
        ins = [torch.randint(0, 1 << 62, (N,), device=dev) for _ in range(args.calib)]
        so = torch.empty(N, dtype=torch.int64, device=dev)
        for _ in range(args.reps):
            K.sum_u64(ins, so)
        torch.cuda.synchronize()
        del ins
    out = []
    for cs in cases:
        t = sorted(cs["times"])
        ms = t[len(t) // 2]
        draws = (len(cs["plan"].pairs) + len(cs["plan"].cross)) * N
        out.append({"C": cs["C"], "W": cs["W"], "L": cs["L"], "ms_median": ms, "ms_min": t[0],
                    "draws_per_s": draws / (ms / 1e3), "local_grad_elems_per_s": cs["L"] * N / (ms / 1e3),
                    "hbm_GBps": (4 * cs["L"] * N + 8 * N) / (ms / 1e3) / 1e9})
    print(json.dumps({"lib": os.environ.get("SFL_SA_LIB", "default"), "elems": N, "cases": out}))


if __name__ == "__main__":
    main()
