#!/usr/bin/env python3
"""Probe of the first launches' ramp: per-launch durations of
the 8-client launch in one process -- 30 launches, 1 s idle, 30 more, then
fresh buffers and 30 more -- to tell an idle-GPU clock ramp from a
first-launches-of-the-process effect."""
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch

    from bench import pair_seed
    from sfl_amd import kernels as K
    from sfl_amd.parallel_sum import plan_generators, plan_rank

    dev = torch.device("cuda", 0)
    N = 100_000_000
    plan = plan_rank([f"client{c}" for c in range(8)], 1, 0)
    pg, ps, cross = plan_generators(plan, pair_seed)

    def bufs():
        xs = [torch.randn(N, device=dev) * 1e-2 for _ in range(8)]
        return xs, torch.zeros(N, dtype=torch.int64, device=dev)

    def batch(xs, s, k=30):
        ev = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(k)]
        for a, b in ev:
            a.record()
            K.fused_clients(xs, [1.0] * 8, pg, ps, cross, 0, s)
            b.record()
        torch.cuda.synchronize()
        return [round(a.elapsed_time(b), 3) for a, b in ev]

    xs, s = bufs()
    torch.cuda.synchronize()
    out = {"first": batch(xs, s)}
    time.sleep(1.0)
    out["after_1s_idle"] = batch(xs, s)
    del xs, s
    xs, s = bufs()
    torch.cuda.synchronize()
    out["fresh_buffers"] = batch(xs, s)
    # 1 s idle, then ~100 ms of other GPU load in this process right before
    # the batch: does preceding load (not this kernel) remove the ramp?
    time.sleep(1.0)
    t = torch.empty(100_000_000, device=dev)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(60):
        t.mul_(1.0000001)
    e1.record()
    out["after_1s_idle_then_load"] = batch(xs, s)
    out["load_ms"] = round(e0.elapsed_time(e1), 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
