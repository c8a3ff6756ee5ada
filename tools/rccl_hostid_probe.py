#!/usr/bin/env python3
"""Probe: real multi-rank RCCL collectives on ONE GPU.

RCCL refuses two ranks on one GPU of one host ("Duplicate GPU detected",
tools/rccl_two_ranks_one_gpu.py): the check compares (host hash, bus id).
With a distinct NCCL_HOSTID per rank every rank looks like its own node, so
RCCL builds the communicator with its network transport (sockets over the
loopback interface) between the ranks -- the collectives' own code (ring /
tree schedules, grouped send / recv, in-place semantics) runs for real at
world W, only the wire is not xGMI.  Checks every sa_comm_* collective
against the expected values.

usage: python tools/rccl_hostid_probe.py --world W   (starts W rank processes)
"""
import argparse
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def hostid_env(rank: int) -> dict:
    """The per-rank environment: a distinct NCCL_HOSTID, sockets on lo."""
    return {"NCCL_HOSTID": f"sfl-onegpu-rank{rank}", "NCCL_SOCKET_IFNAME": "lo", "NCCL_IB_DISABLE": "1",
            "HSA_ENABLE_IPC_MODE_LEGACY": os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0")}


def rank_main():
    import torch
    import torch.distributed as dist

    from sfl_amd.parallel_sum import RcclComm

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dev = torch.device("cuda", 0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {"rank": rank, "world": world}
    try:
        comm = RcclComm(rank, world, 0)
        n = 1000 * world  # elements per shard x world
        base = torch.arange(n * world, dtype=torch.int64, device=dev)
        # reduce-scatter in place: rank r's shard = sum over ranks p of (base + p * 7) there
        x = base + rank * 7
        shard = n
        comm.reduce_scatter_u64(x, x[rank * shard:(rank + 1) * shard])
        torch.cuda.synchronize()
        want = base[rank * shard:(rank + 1) * shard] * world + 7 * (world * (world - 1) // 2)
        out["reduce_scatter"] = bool(torch.equal(x[rank * shard:(rank + 1) * shard], want))
        # uint64 wrap-around: every rank sends 2^63 + rank -> sum mod 2^64
        y = torch.full((world * 64,), -(1 << 63) + rank, dtype=torch.int64, device=dev)
        comm.reduce_scatter_u64(y, y[rank * 64:(rank + 1) * 64])
        torch.cuda.synchronize()
        want_u = (world * (1 << 63) + world * (world - 1) // 2) % (1 << 64)
        want_i = want_u - (1 << 64) if want_u >> 63 else want_u
        out["reduce_scatter_wraps"] = bool((y[rank * 64:(rank + 1) * 64] == want_i).all())
        # all-to-all: recv slot p = rank p's slot `rank` of its send
        s = torch.arange(n * world, dtype=torch.int64, device=dev) + 10**6 * rank
        r = torch.full_like(s, -1)
        comm.alltoall_u64(s, r)
        torch.cuda.synchronize()
        ok = True
        for p in range(world):
            if p == rank:
                ok &= bool((r[p * n:(p + 1) * n] == -1).all())  # own slot not written
            else:
                ok &= bool(torch.equal(r[p * n:(p + 1) * n],
                                       torch.arange(rank * n, (rank + 1) * n, dtype=torch.int64, device=dev) + 10**6 * p))
        out["alltoall"] = ok
        # gather float64 shards to root 0
        f = torch.full((n,), float(rank) + 0.5, dtype=torch.float64, device=dev)
        g = torch.empty(n * world, dtype=torch.float64, device=dev) if rank == 0 else None
        comm.gather_f64(f, g, root=0)
        torch.cuda.synchronize()
        if rank == 0:
            out["gather"] = all(bool((g[p * n:(p + 1) * n] == p + 0.5).all()) for p in range(world))
        # reduce to root 0 (in place on the others), allreduce
        z = torch.full((n,), rank + 1, dtype=torch.int64, device=dev)
        zr = torch.empty_like(z) if rank == 0 else None
        comm.reduce_u64(z, zr, root=0)
        a = torch.full((n,), 3 * rank, dtype=torch.int64, device=dev)
        ar = torch.empty_like(a)
        comm.allreduce_u64(a, ar)
        torch.cuda.synchronize()
        if rank == 0:
            out["reduce"] = bool((zr == world * (world + 1) // 2).all())
        out["allreduce"] = bool((ar == 3 * world * (world - 1) // 2).all())
        comm.close()
    except Exception as e:  # noqa: BLE001 - the probe reports it
        out["error"] = repr(e)[:600]
    # one write(2) per line: the ranks share the parent's stdout pipe, and a
    # print's text and newline can otherwise interleave with another rank's
    os.write(1, ("PROBE " + json.dumps(out) + "\n").encode())
    dist.destroy_process_group()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--world", type=int, default=2)
    ap.add_argument("--rank-main", action="store_true", help=argparse.SUPPRESS)
    args = ap.parse_args()
    if args.rank_main:
        rank_main()
        return
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    procs = []
    for r in range(args.world):
        env = dict(os.environ, RANK=str(r), WORLD_SIZE=str(args.world), LOCAL_RANK="0",
                   MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), **hostid_env(r))
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__), "--rank-main"], env=env))
    rcs = [p.wait(timeout=240) for p in procs]
    sys.exit(max(rcs))


if __name__ == "__main__":
    main()
