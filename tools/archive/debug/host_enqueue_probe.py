#!/usr/bin/env python3
"""Probe: host time to ENQUEUE one pipelined step of the N > 1 bench
(PipelinedMaskedSum.run, 8 chunks) against the GPU time of that step, on
one GPU at world 1 (RcclComm over a single-rank group).  If enqueueing a
step takes longer than the GPU needs for it, the N = 8 run is host-bound.

usage: python tools/debug/host_enqueue_probe.py [--elems 100000000] [--world-shape 8]
  --world-shape W: the per-rank shape of a W-GPU run (8 clients over W ranks).
"""
import argparse
import json
import os
import sys
import tempfile
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--elems", type=int, default=100_000_000)
    ap.add_argument("--world-shape", type=int, default=8)
    ap.add_argument("--steps", type=int, default=50)
    ap.add_argument("--chunks", type=int, default=8)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist

    from bench import pair_seed
    from sfl_amd import _lib
    from sfl_amd.parallel_sum import PipelinedMaskedSum, RcclComm, plan_generators, plan_rank

    _lib.lib()
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", init_method="file://" + os.path.join(tempfile.mkdtemp(), "s"), rank=0,
                            world_size=1)
    comm = RcclComm(0, 1, 0)
    names = [f"client{c}" for c in range(8)]
    plan = plan_rank(names, args.world_shape, 0)
    n = args.elems
    xs = [torch.randn(n, device=dev) * 1e-2 for _ in plan.clients]
    out = []
    for exchange in ("sharded", "direct", "reduce"):
        pipe = PipelinedMaskedSum(comm, dev, n, args.chunks, exchange=exchange)
        total = args.steps + 5
        gens = [[plan_generators(plan, pair_seed, offset=i * n + lo) for lo, _ in pipe.bounds] for i in range(total)]
        s = torch.zeros(pipe.buffer_len, dtype=torch.int64, device=dev)
        dec = torch.zeros(pipe.buffer_len, dtype=torch.float64, device=dev) if exchange != "reduce" else None

        def step(i):
            pipe.run(xs, [1.0] * len(xs), gens[i], plan.n_cross, s, None, dec=dec, join=False)

        for i in range(5):
            step(i)
        torch.cuda.synchronize()
        # host cost with the GPU idle at the start: the loop returns as soon as
        # everything is enqueued (the queue does not block at these depths)
        t0 = time.perf_counter()
        for i in range(args.steps):
            step(5 + i)
        t_enq = time.perf_counter() - t0
        torch.cuda.synchronize()
        t_all = time.perf_counter() - t0
        out.append({"exchange": exchange, "shape": f"<{len(plan.clients)},{plan.n_cross}>", "chunks": len(pipe.bounds),
                    "host_enqueue_ms_per_step": t_enq * 1e3 / args.steps,
                    "wall_ms_per_step": t_all * 1e3 / args.steps})
        print(json.dumps(out[-1]), flush=True)
        del pipe, gens, s, dec
    comm.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
