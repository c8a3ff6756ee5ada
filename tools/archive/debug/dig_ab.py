#!/usr/bin/env python3
"""A/B: fused 8 x 100M launch with and without per-client digests (hipEvents),
interleaved.  usage: python tools/debug/dig_ab.py [--reps 20] [--rounds 5]"""
import argparse, json, os, sys
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))
os.environ.setdefault("SFL_SA_ALLOW_TUNING_BUILD", "1")


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=20)
    ap.add_argument("--rounds", type=int, default=5)
    args = ap.parse_args()
    import torch
    from bench import pair_seed
    from sfl_amd import kernels as K
    from sfl_amd.parallel_sum import plan_generators, plan_rank
    dev = torch.device("cuda", 0)
    N = 100_000_000
    plan = plan_rank([f"client{c}" for c in range(8)], 1, 0)
    xs = [torch.randn(N, device=dev) * 1e-2 for _ in range(8)]
    pg, ps, cross = plan_generators(plan, pair_seed)
    s = torch.empty(N, dtype=torch.int64, device=dev)
    dig = torch.zeros(8, dtype=torch.int64, device=dev)
    res = {"digests": [], "none": []}
    for _ in range(args.rounds):
        for mode in ("digests", "none"):
            d = dig if mode == "digests" else None
            K.fused_clients(xs, [1.0] * 8, pg, ps, cross, 0, s, digests=d)
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                K.fused_clients(xs, [1.0] * 8, pg, ps, cross, 0, s, digests=d)
            e1.record()
            torch.cuda.synchronize()
            res[mode].append(e0.elapsed_time(e1) / args.reps)
    print(json.dumps({k: sorted(v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
