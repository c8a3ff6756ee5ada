"""The multi-GPU path's host logic on CPU with world_size 2 over gloo.

Each rank takes its block of clients (sfl_amd.parallel_sum.plan_rank), builds
exactly the streams its fused launch would expand (internal pairs once, cross
streams per client), emulates that launch with the oracle (CPU checker), and
the uint64 partial sums are reduced to rank 0 with torch.distributed (the
role RCCL plays on the GPUs).  Rank 0 compares with the oracle's full
server sum: the sharding must lose or double no mask.
"""
import os
import tempfile

import numpy as np
import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _worker(rank, world, init, C, n, q):
    import torch

    from oracle import secagg as o
    from sfl_amd.parallel_sum import client_shard, plan_rank

    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    names = [f"client{c}" for c in range(C)][::-1]  # names not in index order: signs matter
    rng = np.random.default_rng(0)
    xs = [(rng.standard_normal(n) * 1e-2).astype(np.float32) for _ in range(C)]
    seeds = o.seeds_for(names)
    plan = plan_rank(names, world, rank)
    assert plan.clients == client_shard(C, world, rank)
    local = {u: o.quantize(xs[u]).copy() for u in plan.clients}
    for (u, v), s in zip(plan.pairs, plan.pair_signs):
        m = o.mask_stream(seeds[names[u]][names[v]], n)
        local[u] = local[u] + m if s > 0 else local[u] - m
        local[v] = local[v] - m if s > 0 else local[v] + m
    for (u, v, s) in plan.cross:
        m = o.mask_stream(seeds[names[u]][names[v]], n)
        local[u] = local[u] + m if s > 0 else local[u] - m
    ref = o.secure_masked(xs, names, seeds=seeds)
    ok_clients = all(np.array_equal(local[u], ref[u]) for u in plan.clients)
    part = np.zeros(n, dtype=np.uint64)
    for u in plan.clients:
        part += local[u]
    t = torch.from_numpy(part.view(np.int64).copy())
    dist.reduce(t, dst=0, op=dist.ReduceOp.SUM)  # int64 add wraps like uint64
    if rank == 0:
        full = o.server_sum(ref)
        q.put((ok_clients, bool(np.array_equal(t.numpy().view(np.uint64), full))))
    else:
        q.put((ok_clients, True))
    dist.destroy_process_group()


@pytest.mark.parametrize("C", [4, 8])
def test_sharded_masked_sum_world2(C):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = "file://" + os.path.join(tempfile.mkdtemp(prefix="sfl_gloo_"), "store")  # no TCP port to race for
    procs = [ctx.Process(target=_worker, args=(r, 2, init, C, 777, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert all(a for a, _ in res), "per-client masked vectors differ from the oracle"
    assert all(b for _, b in res), "reduced masked sum differs from the oracle"


def test_plan_covers_every_pair_once():
    from sfl_amd.parallel_sum import plan_rank

    for C, W in [(8, 1), (8, 2), (8, 4), (8, 8), (32, 8), (4, 2)]:
        names = [f"p{c}" for c in range(C)]
        seen = {}
        for r in range(W):
            p = plan_rank(names, W, r)
            assert p.n_cross == C - C // W
            for u, v in p.pairs:
                seen[(u, v)] = seen.get((u, v), 0) + 2  # both ends applied in one launch
            for u, v, s in p.cross:
                seen[(min(u, v), max(u, v))] = seen.get((min(u, v), max(u, v)), 0) + 1
                assert s == (1 if names[v] > names[u] else -1)
        assert len(seen) == C * (C - 1) // 2 and all(c == 2 for c in seen.values())


@pytest.mark.parametrize("n,chunks", [(0, 4), (1, 4), (1023, 2), (1024, 2), (50_001, 3), (10**8, 4), (10**8, 7)])
def test_chunk_bounds_cover_and_align(n, chunks):
    from sfl_amd.parallel_sum import chunk_bounds

    b = chunk_bounds(n, chunks)
    assert b[0][0] == 0 and b[-1][1] == n
    assert all(lo % 1024 == 0 for lo, _ in b)
    assert all(b[i][1] == b[i + 1][0] for i in range(len(b) - 1))
    assert len(b) <= max(1, chunks)


@pytest.mark.parametrize("n", [1, 1023, 50_003, 10**6 + 7, 10**8])
@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("chunks", [1, 3, 8])
def test_sharded_server_layout(n, world, chunks):
    """The sharded server's split: per chunk, ``world``
    equal shards tile the chunk exactly (only the last chunk is padded, and
    by less than world x 128 elements), shard starts are 1 KiB aligned, and
    the ranks' decoded ranges cover [0, n) once."""
    from sfl_amd.parallel_sum import chunk_bounds, padded_len, rank_shards, shard_layout

    b = chunk_bounds(n, chunks, align=1024 * world)  # PipelinedMaskedSum's sharded bounds
    lay = shard_layout(b, world)
    for j, ((lo, hi), (lo2, k)) in enumerate(zip(b, lay)):
        assert lo == lo2 and k % 128 == 0
        if j < len(b) - 1:
            assert world * k == hi - lo
        else:
            assert 0 <= world * k - (hi - lo) < world * 128
    assert n <= padded_len(b, world) < n + world * 128
    covered = []
    for r in range(world):
        for a, e in rank_shards(b, world, r, n):
            assert 0 <= a <= e <= n
            covered.append((a, e))
    covered.sort()
    pos = 0
    for a, e in covered:
        if a == e:
            continue
        assert a == pos
        pos = e
    assert pos == n


@pytest.mark.parametrize("n", [0, 1, 1000, 70_001, 10**8])
@pytest.mark.parametrize("world", [1, 2, 3, 8])
def test_element_shard_slices(n, world):
    """Element sharding: the ranks' slices tile [0, n) in rank order, every
    slice starts 512-B aligned and holds at most the gather count k."""
    from sfl_amd.parallel_sum import element_shard

    pos = 0
    for r in range(world):
        e0, m, k = element_shard(n, world, r)
        assert e0 == pos and 0 <= m <= k and k % 128 == 0
        pos += m
    assert pos == n


def _standin_worker(rank, world, init, q):
    import torch

    from bench import HostStandinComm

    dist.init_process_group("gloo", init_method=init, rank=rank, world_size=world)
    comm = HostStandinComm(rank, world)
    rng = np.random.default_rng(100 + rank)
    ok = {}
    k = 1001
    for trial in range(2):  # the second round grows the shared slots
        n = k * world * (trial + 1)
        kk = n // world
        send = torch.from_numpy(rng.integers(-2**62, 2**62, n, dtype=np.int64))
        alls = [None] * world
        dist.all_gather_object(alls, send.numpy().copy())  # the expectation, from gloo itself
        total = np.sum(np.stack(alls).view(np.uint64), axis=0, dtype=np.uint64)
        recv = torch.empty(kk, dtype=torch.int64)
        comm.reduce_scatter_u64(send, recv)
        ok[f"rs{trial}"] = bool(np.array_equal(recv.numpy().view(np.uint64), total[rank * kk:(rank + 1) * kk]))
        got = torch.full((n,), -7, dtype=torch.int64)
        comm.alltoall_u64(send, got)
        exp = np.full(n, -7, dtype=np.int64)
        for p in range(world):
            if p != rank:
                exp[p * kk:(p + 1) * kk] = alls[p][rank * kk:(rank + 1) * kk]
        ok[f"a2a{trial}"] = bool(np.array_equal(got.numpy(), exp))
        s2 = send.clone()
        comm.reduce_u64(s2, None, root=1)
        if rank == 1:
            ok[f"red{trial}"] = bool(np.array_equal(s2.numpy().view(np.uint64), total))
        f = torch.from_numpy(rng.standard_normal(kk))
        fs = [None] * world
        dist.all_gather_object(fs, f.numpy().copy())
        g = torch.empty(world * kk, dtype=torch.float64) if rank == 0 else None
        comm.gather_f64(f, g, root=0)
        if rank == 0:
            ok[f"gat{trial}"] = bool(np.array_equal(g.numpy(), np.concatenate(fs)))
    comm.close()
    q.put((rank, ok))
    dist.destroy_process_group()


@pytest.mark.parametrize("world", [2, 3])
def test_host_standin_comm_matches_the_collectives(world):
    """bench.HostStandinComm (the one-GPU rehearsal's stand-in for RcclComm:
    data and barriers through a shared mapping) gives what the
    collectives it stands in for give: reduce-scatter shards of the uint64
    sum, the alltoall slots (own slot untouched), the in-place uint64
    reduce to a root, the float64 gather -- also after its slots grow."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    init = "file://" + os.path.join(tempfile.mkdtemp(prefix="sfl_gloo_"), "store")
    procs = [ctx.Process(target=_standin_worker, args=(r, world, init, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=30)
    for rank, ok in res:
        assert ok and all(ok.values()), (rank, ok)
