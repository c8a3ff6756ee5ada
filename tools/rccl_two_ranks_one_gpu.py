#!/usr/bin/env python3
"""Probe: can two ranks on ONE GPU form an RCCL communicator (our sa_comm_*)
and run a reduce-scatter?  Run as: torchrun --nproc-per-node 2 ... this file.
Every rank uses cuda:0; prints what RCCL did (or the error it gave)."""
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)


def main():
    import torch
    import torch.distributed as dist

    from sfl_amd.parallel_sum import RcclComm

    rank, world = int(os.environ["RANK"]), int(os.environ["WORLD_SIZE"])
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    out = {"rank": rank}
    try:
        comm = RcclComm(rank, world, 0)
        n = 1 << 20
        x = torch.full((n * world,), rank + 1, dtype=torch.int64, device="cuda:0")
        comm.reduce_scatter_u64(x, x[rank * n:(rank + 1) * n])
        torch.cuda.synchronize()
        out["reduce_scatter_ok"] = bool((x[rank * n:(rank + 1) * n] == sum(range(1, world + 1))).all())
        comm.close()
    except Exception as e:  # noqa: BLE001 - the probe reports it
        out["error"] = repr(e)[:400]
    print(json.dumps(out), flush=True)
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
