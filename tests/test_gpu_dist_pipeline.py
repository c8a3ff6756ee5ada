"""The multi-GPU data path with REAL ranks: W processes, each running its
block of clients through ``PipelinedMaskedSum`` (the bench's chunked fused
launches, the comm stream and its per-chunk events, the in-place reduce) on
the one GPU of the test box.

The exchange is the product's ``RcclComm`` running real RCCL collectives
between the W ranks (kind "rccl": RCCL refuses two ranks on one GPU of one
host, so each rank gets its own NCCL_HOSTID and RCCL connects the "nodes"
through its socket transport on lo -- ``benchkit.standin.one_gpu_rccl_comm``),
and again through the host stand-in with the same contract (kind
"standin"): on the comm stream, after the chunk's event, the partial sum
is reduced to the root IN PLACE (recv=None) -- uint64 addition mod 2^64.
Everything else is the product code path the N > 1 bench runs.  The root's buffer must equal the oracle's server sum bit for bit, and
every client's digest the oracle's."""
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _run_ranks(target, world, args):
    """Spawn ``world`` rank processes and collect one result each.  A stalled
    rank fails the test within 150 s (every worker dumps its Python stacks
    to stderr after 100 s first) instead of running into the GPU harness's
    3-minute silence limit; leftover ranks are killed."""
    import torch.multiprocessing as mp

    import tempfile

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    # file-based rendezvous: no TCP port that another process could take
    # between choosing it and binding it (a rank would then wait forever)
    init = "file://" + os.path.join(tempfile.mkdtemp(prefix="sfl_ranks_"), "store")
    procs = [ctx.Process(target=_with_dump, args=(target, r, world, init, *args, q)) for r in range(world)]
    for p in procs:
        p.start()
    try:
        return sorted(q.get(timeout=150) for _ in procs)
    finally:
        for p in procs:
            p.join(timeout=30)
            if p.is_alive():
                p.kill()


def _with_dump(target, *args):
    import faulthandler
    import sys

    faulthandler.dump_traceback_later(100, exit=False, file=sys.stderr)
    target(*args)


def _comm(kind, rank, world):
    """The exchange under test: the product's RcclComm with the ranks made
    distinct RCCL nodes on the one GPU (real RCCL collectives over its socket
    transport), or the host stand-in."""
    from benchkit.standin import HostStandinComm, one_gpu_rccl_comm

    return one_gpu_rccl_comm(rank, world) if kind == "rccl" else HostStandinComm(rank, world)


def _worker(rank, world, init, n, chunks, offset, kind, q):
    import torch
    import torch.distributed as dist

    from oracle import secagg as o
    from sfl_amd.parallel_sum import PipelinedMaskedSum, plan_generators, plan_rank

    try:
        dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
        C = 8
        names = [f"client{c}" for c in range(C)]
        seeds = o.seeds_for(names)
        seed_of = lambda u, v: seeds[names[u]][names[v]]  # noqa: E731
        rng = np.random.default_rng(77)
        xs = [(rng.standard_normal(n) * 1e-2).astype(np.float32) for _ in range(C)]
        dev = torch.device("cuda", 0)
        plan = plan_rank(names, world, rank)
        pipe = PipelinedMaskedSum(_comm(kind, rank, world), dev, n, chunks)
        gens = [plan_generators(plan, seed_of, offset=offset + lo) for lo, _ in pipe.bounds]
        part = torch.empty(n, dtype=torch.int64, device=dev)
        dig = torch.zeros(len(plan.clients), dtype=torch.int64, device=dev)
        flags = torch.zeros(1, dtype=torch.int32, device=dev)
        pipe.run([torch.from_numpy(xs[c]).to(dev) for c in plan.clients], [1.0] * len(plan.clients), gens,
                 plan.n_cross, part, None, digests=dig, flags=flags)
        torch.cuda.synchronize()
        masked = o.secure_masked(xs, names, seeds=seeds, offset=offset)
        dig_ok = [int(d) for d in dig.cpu().numpy().view(np.uint64)] == [o.digest(masked[c]) for c in plan.clients]
        sum_ok = True
        if rank == 0:
            sum_ok = bool(np.array_equal(part.cpu().numpy().view(np.uint64), o.server_sum(masked)))
        q.put((rank, dig_ok, sum_ok, int(flags.item())))
        dist.destroy_process_group()
    except BaseException as e:  # noqa: BLE001 - reported to the parent
        q.put((rank, repr(e), False, -1))


@pytest.mark.parametrize("kind", ["rccl", "standin"])
@pytest.mark.parametrize("world,chunks", [(2, 4), (4, 3), (8, 8)])
def test_ranks_pipeline_and_in_place_reduce(world, chunks, kind):
    if torch.cuda.device_count() == 0:  # asked without initialising HIP here (conftest: this module runs early)
        pytest.skip("no GPU")
    res = _run_ranks(_worker, world, (50_003, chunks, 10**9 + 5, kind))
    for rank, dig_ok, sum_ok, fl in res:
        assert dig_ok is True, (rank, dig_ok)
        assert sum_ok, f"rank {rank}: root's in-place reduced sum differs from the oracle"
        assert fl == 0


def _worker_sharded(rank, world, init, n, chunks, offset, exchange, kind, q):
    import torch
    import torch.distributed as dist

    from oracle import secagg as o
    from sfl_amd.parallel_sum import PipelinedMaskedSum, plan_generators, plan_rank, rank_shards

    try:
        dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
        C = 8
        names = [f"client{c}" for c in range(C)]
        seeds = o.seeds_for(names)
        seed_of = lambda u, v: seeds[names[u]][names[v]]  # noqa: E731
        rng = np.random.default_rng(78)
        xs = [(rng.standard_normal(n) * 1e-2).astype(np.float32) for _ in range(C)]
        dev = torch.device("cuda", 0)
        plan = plan_rank(names, world, rank)
        pipe = PipelinedMaskedSum(_comm(kind, rank, world), dev, n, chunks, exchange=exchange)
        gens = [plan_generators(plan, seed_of, offset=offset + lo) for lo, _ in pipe.bounds]
        part = torch.zeros(pipe.buffer_len, dtype=torch.int64, device=dev)
        dec = torch.zeros(pipe.buffer_len, dtype=torch.float64, device=dev)
        pipe.run([torch.from_numpy(xs[c]).to(dev) for c in plan.clients], [1.0] * len(plan.clients), gens,
                 plan.n_cross, part, None, dec=dec, gather=True)
        torch.cuda.synchronize()
        ssum = o.server_sum(o.secure_masked(xs, names, seeds=seeds, offset=offset))
        want = o.decode(ssum)
        got_s, got_d = part.cpu().numpy().view(np.uint64), dec.cpu().numpy()
        shard_ok = all(np.array_equal(got_s[a:b], ssum[a:b]) and np.array_equal(got_d[a:b], want[a:b])
                       for a, b in rank_shards(pipe.bounds, world, rank, n))
        full_ok = bool(np.array_equal(got_d[:n], want)) if rank == 0 else True
        q.put((rank, shard_ok, full_ok))
        dist.destroy_process_group()
    except BaseException as e:  # noqa: BLE001 - reported to the parent
        q.put((rank, repr(e), False))


@pytest.mark.parametrize("kind", ["rccl", "standin"])
@pytest.mark.parametrize("exchange", ["sharded", "direct"])
@pytest.mark.parametrize("world,chunks", [(2, 3), (4, 2), (8, 8)])
def test_ranks_sharded_server(world, chunks, exchange, kind):
    """exchange="sharded" (reduce-scatter) or "direct" (shard transfers +
    a local sum_u64 through the staging buffer) with W real ranks: every
    rank's shard of the masked sum and its float64 decode equal the oracle's
    on that range, and the root's gathered decode equals the oracle's whole
    decoded sum."""
    if torch.cuda.device_count() == 0:  # asked without initialising HIP here (conftest: this module runs early)
        pytest.skip("no GPU")
    res = _run_ranks(_worker_sharded, world, (70_001, chunks, 3 * 10**9 + 1, exchange, kind))
    for rank, shard_ok, full_ok in res:
        assert shard_ok is True, (rank, shard_ok)
        assert full_ok, f"rank {rank}: gathered decode differs from the oracle"
