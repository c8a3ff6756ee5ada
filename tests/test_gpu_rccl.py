"""Our RCCL communicator (sa_comm_*) on one MI355X: world size 1 exercises
init / reduce / allreduce / destroy through the C-ABI (multi-rank runs need
the 8-GPU node the driver uses; the sharding logic is covered by gloo tests)."""
import os
import socket

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def test_rccl_world1_reduce_is_identity():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.distributed as dist

    from sfl_amd.parallel_sum import RcclComm

    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=0, world_size=1)
    try:
        comm = RcclComm(0, 1, 0)
        rng = np.random.default_rng(1)
        a = rng.integers(0, 2**64 - 1, 100_003, dtype=np.uint64)
        send = torch.from_numpy(a.view(np.int64).copy()).cuda()
        recv = torch.empty_like(send)
        comm.reduce_u64(send, recv, root=0)
        recv2 = torch.empty_like(send)
        comm.allreduce_u64(send, recv2)
        torch.cuda.synchronize()
        assert torch.equal(recv, send) and torch.equal(recv2, send)
        comm.close()
    finally:
        dist.destroy_process_group()
