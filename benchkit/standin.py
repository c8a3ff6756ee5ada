"""The one-GPU rehearsal's communicators (bench.py --rehearse-one-gpu;
tests/test_gpu_dist_pipeline.py): real RCCL between ranks that share the
GPU (``one_gpu_rccl_comm``, the default) or the host stand-in
(``HostStandinComm``)."""

from __future__ import annotations

import os
import time


def one_gpu_rccl_env(rank: int) -> dict:
    """The environment that lets W ranks on ONE GPU form a real RCCL
    communicator: RCCL refuses two ranks on one device of one host
    ("Duplicate GPU detected", a (host hash, bus id) check), and NCCL_HOSTID
    sets the host hash -- a distinct id per rank makes every rank its own
    "node", so RCCL connects them through its network transport (sockets on
    the loopback interface) and runs its collectives' own schedules at world
    W (tools/rccl_hostid_probe.py; profiles/r05/rccl_hostid_w*.log).  Only
    the wire differs from the node's xGMI."""
    return {"NCCL_HOSTID": f"sfl-onegpu-rank{rank}", "NCCL_SOCKET_IFNAME": "lo", "NCCL_IB_DISABLE": "1"}


def one_gpu_rccl_comm(rank: int, world: int, group=None):
    """The product's ``RcclComm`` for a rank of a one-GPU rehearsal (every
    rank on device 0), after ``one_gpu_rccl_env``; the unique id travels
    through the torch.distributed ``group`` (gloo) as on the node."""
    os.environ.update(one_gpu_rccl_env(rank))
    from sfl_amd.parallel_sum import RcclComm

    return RcclComm(rank, world, 0, group)


class HostStandinComm:
    """--rehearse-one-gpu only: RcclComm's contract (reduce_u64,
    reduce_scatter_u64, alltoall_u64, gather_f64) for N rank processes on
    ONE GPU (RCCL refuses two ranks on one device: "Duplicate GPU detected"),
    so every design's code path runs.  Everything moves through memory shared
    by the ranks on this host: every rank writes its host copy of the send
    buffer into its slot, a barrier, every rank reads what the collective
    gives it, a second barrier before the slots are reused.  The barrier is
    in the shared memory too (each rank publishes an epoch in its own cache
    line and waits for every rank's), so the data path touches no socket:
    round 4's W = 8 rehearsals now and then sat for 30-50 s inside one gloo
    all_reduce / barrier on every rank at once.  gloo only
    sets the mappings up.  Called on the comm stream like RcclComm;
    ``send.cpu()`` waits for the chunk's launch.  Its timings are host
    copies, not xGMI: a rehearsal checks the N > 1 control flow, never the
    rate."""

    def __init__(self, rank: int, world: int, group=None):
        import tempfile
        import uuid

        import numpy as np
        import torch.distributed as dist

        self.rank, self.world, self.group = rank, world, group
        # /dev/shm keeps the slots in memory (a disk-backed /tmp file made the
        # full-size W = 8 rehearsal write back GBs per step); each file is
        # unlinked as soon as every rank has mapped it, so nothing is left
        # behind however a rank ends
        base = "/dev/shm" if os.access("/dev/shm", os.W_OK) else tempfile.gettempdir()
        box = [os.path.join(base, f"sfl_rehearsal_{os.getpid()}_{uuid.uuid4().hex[:12]}") if rank == 0 else None]
        dist.broadcast_object_list(box, src=0, group=group)
        self.prefix, self.cap, self.gen, self.mm, self.epoch = box[0], 0, 0, None, 0
        self.ctl = self._shared((world, 8), np.int64)  # [r, 0]: rank r's barrier epoch

    def _shared(self, shape, dtype):
        """A new zeroed mapping of ``shape`` shared by every rank (collective)."""
        import numpy as np
        import torch.distributed as dist

        path = f"{self.prefix}_{self.gen}"
        self.gen += 1
        if self.rank == 0:
            with open(path, "wb") as f:
                f.truncate(int(np.prod(shape)) * np.dtype(dtype).itemsize)
        dist.barrier(group=self.group)
        mm = np.memmap(path, dtype=dtype, mode="r+", shape=shape)
        dist.barrier(group=self.group)
        if self.rank == 0:
            os.unlink(path)  # the mappings keep the pages until every rank drops them
        return mm

    def _barrier(self):
        """Every rank has reached the same epoch.  Each rank's epoch word has
        one writer; x86 keeps stores in order, so a rank that sees another's
        epoch also sees the slot bytes that rank wrote before it."""
        self.epoch += 1
        self.ctl[self.rank, 0] = self.epoch
        col = self.ctl[:, 0]
        spins = 0
        while int(col.min()) < self.epoch:
            spins += 1
            time.sleep(0 if spins < 200 else 50e-6)

    def _slots(self, nbytes: int):
        """The (world, cap) byte view of the shared slots, grown (collectively:
        every rank asks for the same size) when an op needs more."""
        import numpy as np

        if nbytes > self.cap:
            self.cap = max(nbytes, 2 * self.cap)
            self.mm = None
            self.mm = self._shared((self.world, self.cap), np.uint8)
        return self.mm

    def _post(self, t):
        """This rank's host copy of ``t`` into its slot; then every rank's slots
        are readable.  Returns (slots, nbytes)."""
        import numpy as np

        host = t.cpu().numpy()  # on the comm stream: waits for the chunk's launch
        nb = host.nbytes
        mm = self._slots(nb)
        mm[self.rank, :nb] = host.reshape(-1).view(np.uint8)  # a shared mapping: no msync needed between processes
        self._barrier()
        return mm, nb

    def reduce_u64(self, send, recv, root: int = 0):
        import numpy as np
        import torch

        mm, nb = self._post(send)
        if self.rank == root:
            total = np.sum(mm[:, :nb].view(np.uint64), axis=0, dtype=np.uint64)  # wraps mod 2^64
            (recv if recv is not None else send).copy_(torch.from_numpy(total.view(np.int64)))
        self._barrier()
        return recv

    def reduce_scatter_u64(self, send, recv):
        import numpy as np
        import torch

        if send.numel() != recv.numel() * self.world:
            raise ValueError("reduce_scatter: shard sizes")
        mm, nb = self._post(send)
        k = recv.numel()
        part = mm[:, :nb].view(np.uint64)[:, self.rank * k:(self.rank + 1) * k]
        recv.copy_(torch.from_numpy(np.sum(part, axis=0, dtype=np.uint64).view(np.int64)))
        self._barrier()
        return recv

    def alltoall_u64(self, send, recv):
        import numpy as np
        import torch

        mm, nb = self._post(send)
        k = send.numel() // self.world
        slots = mm[:, :nb].view(np.int64)
        for p in range(self.world):
            if p != self.rank:
                recv[p * k:(p + 1) * k].copy_(torch.from_numpy(np.array(slots[p, self.rank * k:(self.rank + 1) * k])))
        self._barrier()
        return recv

    def gather_f64(self, send, recv, root: int = 0):
        import numpy as np
        import torch

        mm, nb = self._post(send)
        if self.rank == root:
            recv.copy_(torch.from_numpy(np.array(mm[:, :nb].view(np.float64)).reshape(-1)))
        self._barrier()
        return recv

    def close(self):
        self.mm = None  # the slot files are unlinked already: dropping the mapping frees them
        self._barrier()
