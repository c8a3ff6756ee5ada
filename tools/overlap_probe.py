#!/usr/bin/env python3
"""Does the pipelined exchange overlap the masking?  One-GPU probe of the
N > 1 pipeline.

bench.py's N > 1 step is PipelinedMaskedSum: chunk j's masking launch on the
compute stream while chunk j-1's exchange runs on a comm stream.  The masking
grid is occupancy-sized (it fills every CU), so an exchange KERNEL (RCCL's)
queued behind it may not start until the masking launch drains.  No
multi-GPU box is ours, so this probe runs the bench's pipeline for one
rank's shape on one GPU with a stand-in communicator whose reduce-scatter
launches tools/microbench/libspin.so's k_spin (B resident workgroups for U
microseconds, no memory traffic: a few-CU, link-bound kernel like RCCL's)
and times, per step:

  mask   the masking alone (no exchange),
  spin   the stand-in exchange alone (8 chunks of U us),
  both   the pipeline with both,

for each sa_set_masking_reserve value (CUs of the masking grid left free).
Perfect overlap: both ~ max(mask, spin) + one chunk; none: mask + spin.

usage: python tools/overlap_probe.py [--world 8] [--elems 100000000] [--blocks 16] [--usec 200]
       [--reserve 0,4,8,16] [--steps 20]
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


class SpinComm:
    """RcclComm's reduce_scatter_u64 contract, doing no data movement: it
    launches k_spin on the current (comm) stream."""

    def __init__(self, world, rank, blocks, usec):
        self.world, self.rank, self.blocks, self.usec = world, rank, blocks, usec
        self.lib = C.CDLL(os.path.join(ROOT, "tools", "microbench", "libspin.so"))
        self.lib.spin_launch.argtypes = [C.c_int, C.c_double, C.c_void_p]

    def reduce_scatter_u64(self, send, recv):
        import torch

        s = torch.cuda.current_stream(send.device).cuda_stream
        if self.lib.spin_launch(self.blocks, self.usec, C.c_void_p(s)):
            raise RuntimeError("spin_launch failed")
        return recv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--elems", type=int, default=100_000_000)
    ap.add_argument("--blocks", type=int, default=16)
    ap.add_argument("--usec", type=float, default=200.0)
    ap.add_argument("--reserve", default="0,4,8,16")
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    args = ap.parse_args()
    import torch

    from bench import pair_seed
    from sfl_amd import _lib as L
    from sfl_amd.parallel_sum import PipelinedMaskedSum, plan_generators, plan_rank

    L.lib()
    dev = torch.device("cuda", 0)
    names = [f"client{c}" for c in range(args.clients)]
    plan = plan_rank(names, args.world, 0)
    Lc, N = len(plan.clients), args.elems
    xs = [torch.randn(N, device=dev) * 1e-2 for _ in range(Lc)]
    comm = SpinComm(args.world, 0, args.blocks, args.usec)

    def make(with_comm):
        pipe = PipelinedMaskedSum(comm if with_comm else None, dev, N, 8, exchange="sharded" if with_comm else "reduce")
        gens = [plan_generators(plan, pair_seed, offset=lo) for lo, _ in pipe.bounds]
        sb = torch.zeros(pipe.buffer_len, dtype=torch.int64, device=dev)
        dec = torch.zeros(pipe.buffer_len, dtype=torch.float64, device=dev) if with_comm else None
        return lambda: pipe.run(xs, [1.0] * Lc, gens, plan.n_cross, sb, None, join=False, dec=dec)

    def spin_only():
        s = torch.cuda.current_stream(dev).cuda_stream
        for _ in range(8):
            comm.lib.spin_launch(args.blocks, args.usec, C.c_void_p(s))

    def timeit(fn):
        for _ in range(args.warmup):
            fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) * 1e3 / args.steps

    out = {"world": args.world, "local_clients": Lc, "cross": plan.n_cross, "elems": N, "blocks": args.blocks,
           "usec_per_chunk": args.usec, "chunks": 8, "spin_ms": timeit(spin_only), "by_reserve": []}
    run_mask, run_both = make(False), make(True)
    for r in [int(v) for v in args.reserve.split(",")]:
        L.check(L.lib().sa_set_masking_reserve(r), "sa_set_masking_reserve")
        m, b = timeit(run_mask), timeit(run_both)
        out["by_reserve"].append({"reserve_cus": r, "mask_ms": m, "both_ms": b,
                                  "perfect_overlap_ms": max(m, out["spin_ms"]) + max(m, out["spin_ms"]) / 8,
                                  "no_overlap_ms": m + out["spin_ms"]})
    L.check(L.lib().sa_set_masking_reserve(0), "sa_set_masking_reserve")
    print(json.dumps(out), flush=True)


if __name__ == "__main__":
    main()
