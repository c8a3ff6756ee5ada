#!/usr/bin/env python3
"""Diagnostic: does an RCCL communicator created (and destroyed) in a parent
process stall W spawned rank processes that then share the GPU?  Reproduces
the order in which tests/test_gpu_rccl.py runs before
tests/test_gpu_dist_pipeline.py; every worker dumps its Python stacks after
--dump seconds so a stall shows where it waits.

usage: python tools/debug/rccl_then_spawn.py [--world 8] [--rccl-first 1] [--dump 60]
"""
import argparse
import faulthandler
import os
import socket
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def worker(rank, world, port, dump, q):
    faulthandler.dump_traceback_later(dump, exit=False, file=sys.stderr)
    t0 = time.time()
    import test_gpu_dist_pipeline as T

    T._worker(rank, world, port, 50_003, 8, 10**9 + 5, q)
    print(f"rank {rank} done in {time.time() - t0:.1f} s", file=sys.stderr, flush=True)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=8)
    ap.add_argument("--rccl-first", type=int, default=1)
    ap.add_argument("--dump", type=float, default=60.0)
    args = ap.parse_args()
    import torch
    import torch.distributed as dist
    import torch.multiprocessing as mp

    if args.rccl_first:
        from sfl_amd.parallel_sum import RcclComm

        os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(_port()))
        dist.init_process_group("gloo", rank=0, world_size=1)
        c = RcclComm(0, 1, 0)
        x = torch.ones(1024, dtype=torch.int64, device="cuda")
        c.reduce_u64(x, x)
        torch.cuda.synchronize()
        c.close()
        dist.destroy_process_group()
        print("parent: RCCL comm created, used and destroyed", file=sys.stderr, flush=True)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _port()
    t0 = time.time()
    procs = [ctx.Process(target=worker, args=(r, args.world, port, args.dump, q)) for r in range(args.world)]
    for p in procs:
        p.start()
    try:
        res = sorted(q.get(timeout=args.dump + 60) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=5)
            if p.is_alive():
                p.kill()
    print(f"all {args.world} ranks returned in {time.time() - t0:.1f} s: {res}", flush=True)


if __name__ == "__main__":
    main()
