"""Our RCCL communicator (sa_comm_*) on one MI355X: world size 1 exercises
init / reduce / allreduce / destroy through the C-ABI, and the pipelined
masking + reduce of one rank (multi-rank runs need the 8-GPU node the driver
uses; the sharding logic is covered by gloo tests)."""
import json
import os
import subprocess
import sys
import tempfile

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def comm():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    import torch.distributed as dist

    from sfl_amd.parallel_sum import RcclComm

    # a file-store rendezvous: no port to probe (and race for)
    fd, path = tempfile.mkstemp(prefix="sfl_rccl_store_")
    os.close(fd)
    os.unlink(path)
    dist.init_process_group("gloo", store=dist.FileStore(path, 1), rank=0, world_size=1)
    c = RcclComm(0, 1, 0)
    yield c
    c.close()
    dist.destroy_process_group()
    if os.path.exists(path):
        os.unlink(path)


def test_rccl_world1_reduce_is_identity(comm):
    rng = np.random.default_rng(1)
    a = rng.integers(0, 2**64 - 1, 100_003, dtype=np.uint64)
    send = torch.from_numpy(a.view(np.int64).copy()).cuda()
    recv = torch.empty_like(send)
    comm.reduce_u64(send, recv, root=0)
    recv2 = torch.empty_like(send)
    comm.allreduce_u64(send, recv2)
    torch.cuda.synchronize()
    assert torch.equal(recv, send) and torch.equal(recv2, send)


@pytest.mark.parametrize("chunks", [1, 3, 7])
def test_pipelined_masked_sum_matches_oracle(comm, chunks):
    """Rank 0 of 8 clients over 2 GPUs (4 local clients + 4 cross streams
    each), masking of chunk j overlapped with the reduce of chunk j-1: equals
    the oracle's sum of those clients' masked vectors, bit for bit."""
    from oracle import secagg as o
    from sfl_amd.parallel_sum import PipelinedMaskedSum, plan_generators, plan_rank

    C, W, n, offset = 8, 2, 50_001, 123
    names = [f"client{c}" for c in range(C)]
    seeds = o.seeds_for(names)
    plan = plan_rank(names, W, 0)
    rng = np.random.default_rng(chunks)
    xs = [(rng.standard_normal(n) * 1e-2).astype(np.float32) for _ in range(C)]
    masked = o.secure_masked(xs, names, seeds=seeds, offset=offset)
    exp = np.zeros(n, dtype=np.uint64)
    for c in plan.clients:
        exp += masked[c]
    dev = torch.device("cuda", 0)
    pipe = PipelinedMaskedSum(comm, dev, n, chunks)
    seed_of = lambda u, v: seeds[names[u]][names[v]]  # noqa: E731
    gens = [plan_generators(plan, seed_of, offset=offset + lo) for lo, _ in pipe.bounds]
    s = torch.empty(n, dtype=torch.int64, device=dev)
    recv = torch.empty(n, dtype=torch.int64, device=dev)
    dig = torch.zeros(len(plan.clients), dtype=torch.int64, device=dev)
    kev = []
    pipe.run([torch.from_numpy(xs[c]).to(dev) for c in plan.clients], [1.0] * len(plan.clients), gens,
             plan.n_cross, s, recv, digests=dig, kernel_events=kev)
    torch.cuda.synchronize()
    assert len(kev) == len(pipe.bounds)
    assert np.array_equal(recv.cpu().numpy().view(np.uint64), exp)
    assert [int(v) for v in dig.cpu().numpy().view(np.uint64)] == [o.digest(masked[c]) for c in plan.clients]


def test_back_to_back_rounds_without_join(comm):
    """bench.py's form: rounds run back to back with join=False, so a round's
    reduces may still be reading the shared partial-sum buffer when the next
    round's launches start; each chunk's launch waits for that chunk's
    previous reduce, so every round's received sum equals the oracle's."""
    from oracle import secagg as o
    from sfl_amd.parallel_sum import PipelinedMaskedSum, plan_generators, plan_rank

    C, W, n, chunks = 8, 2, 40_003, 5
    names = [f"client{c}" for c in range(C)]
    seeds = o.seeds_for(names)
    plan = plan_rank(names, W, 0)
    dev = torch.device("cuda", 0)
    pipe = PipelinedMaskedSum(comm, dev, n, chunks)
    seed_of = lambda u, v: seeds[names[u]][names[v]]  # noqa: E731
    s = torch.empty(n, dtype=torch.int64, device=dev)
    exps, recvs = [], []
    for r in range(3):
        rng = np.random.default_rng(100 + r)
        xs = [(rng.standard_normal(n) * 1e-2).astype(np.float32) for _ in range(C)]
        masked = o.secure_masked(xs, names, seeds=seeds, offset=r * n)
        exp = np.zeros(n, dtype=np.uint64)
        for c in plan.clients:
            exp += masked[c]
        exps.append(exp)
        gens = [plan_generators(plan, seed_of, offset=r * n + lo) for lo, _ in pipe.bounds]
        recvs.append(torch.empty(n, dtype=torch.int64, device=dev))
        pipe.run([torch.from_numpy(xs[c]).to(dev) for c in plan.clients], [1.0] * len(plan.clients), gens,
                 plan.n_cross, s, recvs[-1], join=False)
    torch.cuda.synchronize()
    for r in range(3):
        assert np.array_equal(recvs[r].cpu().numpy().view(np.uint64), exps[r]), r


def test_rccl_world1_reduce_scatter_and_gather(comm):
    """The sharded server's collectives at world 1: the reduce-scatter of one
    shard is the identity (in place and out of place), the gather a copy."""
    rng = np.random.default_rng(2)
    a = rng.integers(0, 2**64 - 1, 70_001, dtype=np.uint64)
    send = torch.from_numpy(a.view(np.int64).copy()).cuda()
    out = torch.empty_like(send)
    comm.reduce_scatter_u64(send, out)
    comm.reduce_scatter_u64(send, send)  # in place
    f = torch.from_numpy(rng.standard_normal(70_001)).cuda()
    g = torch.empty_like(f)
    comm.gather_f64(f, g, root=0)
    torch.cuda.synchronize()
    assert torch.equal(out, send) and torch.equal(send.cpu(), torch.from_numpy(a.view(np.int64)))
    assert torch.equal(g, f)


def test_rccl_world1_alltoall_leaves_own_slot(comm):
    """sa_comm_alltoall_u64 at world 1: no peer, so nothing moves and the
    receive buffer's own slot is left untouched."""
    send = torch.arange(4099, dtype=torch.int64, device="cuda")
    recv = torch.full_like(send, -7)
    comm.alltoall_u64(send, recv)
    torch.cuda.synchronize()
    assert bool((recv == -7).all())


@pytest.mark.parametrize("exchange", ["sharded", "direct"])
@pytest.mark.parametrize("chunks", [1, 3])
def test_sharded_server_pipeline_world1(comm, chunks, exchange):
    """exchange="sharded" at world 1 (the whole vector is rank 0's shard):
    8 co-located clients, every chunk reduce-scattered, decoded on the comm
    stream and gathered, two rounds back to back (join=False); the decoded
    result equals the oracle's decode of the server sum bit for bit."""
    from oracle import secagg as o
    from sfl_amd.parallel_sum import PipelinedMaskedSum, plan_generators, plan_rank

    C, n = 8, 60_007
    names = [f"client{c}" for c in range(C)]
    seeds = o.seeds_for(names)
    plan = plan_rank(names, 1, 0)
    dev = torch.device("cuda", 0)
    pipe = PipelinedMaskedSum(comm, dev, n, chunks, exchange=exchange)
    assert pipe.buffer_len >= n
    seed_of = lambda u, v: seeds[names[u]][names[v]]  # noqa: E731
    s = torch.zeros(pipe.buffer_len, dtype=torch.int64, device=dev)
    decs, exps = [], []
    for r in range(2):
        rng = np.random.default_rng(300 + r)
        xs = [(rng.standard_normal(n) * 1e-2).astype(np.float32) for _ in range(C)]
        exps.append(o.decode(o.server_sum(o.secure_masked(xs, names, seeds=seeds, offset=r * n)), divisor=4.0))
        gens = [plan_generators(plan, seed_of, offset=r * n + lo) for lo, _ in pipe.bounds]
        decs.append(torch.empty(pipe.buffer_len, dtype=torch.float64, device=dev))
        pipe.run([torch.from_numpy(x).to(dev) for x in xs], [1.0] * C, gens, plan.n_cross, s, None,
                 dec=decs[-1], divisor=4.0, gather=True, join=False)
    torch.cuda.synchronize()
    for r in range(2):
        assert np.array_equal(decs[r][:n].cpu().numpy(), exps[r]), r


@pytest.mark.parametrize("exchange", ["reduce", "sharded", "direct"])
def test_pipelined_world1_at_1m_matches_oracle_server_sum(comm, exchange):
    """bench.py --gpus 1 --dist's data path at n = 1,000,003: 8 co-located
    clients, the bench's 8-chunk pipeline through RcclComm (ncclReduce in
    place to the root, or the sharded server's ncclReduceScatter + decode),
    round 2's stream positions; the root's masked sum equals the oracle's
    server_sum bit for bit, and the sharded decode the oracle's decode."""
    from oracle import secagg as o
    from sfl_amd.parallel_sum import PipelinedMaskedSum, plan_generators, plan_rank

    C, n, rnd = 8, 1_000_003, 2
    names = [f"client{c}" for c in range(C)]
    seeds = o.seeds_for(names)
    plan = plan_rank(names, 1, 0)
    rng = np.random.default_rng(4242)
    xs = [(rng.standard_normal(n) * 1e-2).astype(np.float32) for _ in range(C)]
    exp = o.server_sum(o.secure_masked(xs, names, seeds=seeds, offset=rnd * n))
    dev = torch.device("cuda", 0)
    pipe = PipelinedMaskedSum(comm, dev, n, 8, exchange=exchange)
    assert len(pipe.bounds) == 8
    seed_of = lambda u, v: seeds[names[u]][names[v]]  # noqa: E731
    gens = [plan_generators(plan, seed_of, offset=rnd * n + lo) for lo, _ in pipe.bounds]
    s = torch.zeros(pipe.buffer_len, dtype=torch.int64, device=dev)
    dec = torch.zeros(pipe.buffer_len, dtype=torch.float64, device=dev) if exchange != "reduce" else None
    flags = torch.zeros(1, dtype=torch.int32, device=dev)
    pipe.run([torch.from_numpy(x).to(dev) for x in xs], [1.0] * C, gens, plan.n_cross, s, None, flags=flags,
             dec=dec)
    torch.cuda.synchronize()
    assert int(flags.item()) == 0
    assert np.array_equal(s[:n].cpu().numpy().view(np.uint64), exp)
    if dec is not None:
        assert np.array_equal(dec[:n].cpu().numpy(), o.decode(exp))


ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def bench_variants():
    sys.path.insert(0, ROOT)
    import bench

    return bench.VARIANTS


@pytest.mark.parametrize("opts", [["--exchange", "reduce"], ["--exchange", "sharded", "--gather"]])
def test_bench_self_launched_dist_world1(opts):
    """The driver's N>1 bench path on this box's one GPU: `bench.py --gpus 1
    --dist` starts torchrun as a child process (not an exec), whose rank runs
    init_process_group("nccl") -> RcclComm -> the pipelined exchange, then
    times every other design in the same process group.  One JSON line,
    n_gpus 1, the exchange and all five designs reported."""
    env = dict(os.environ)
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--dist", "--elems",
                        "1000003", "--steps", "3", "--warmup", "1", "--variant-steps", "2",
                        "--cpu-baseline-seconds", "0", "--watchdog-seconds", "100", *opts],
                       capture_output=True, text=True, timeout=110, env=env, cwd=ROOT)
    assert r.returncode == 0, (r.stdout[-2000:], r.stderr[-3000:])
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert line["n_gpus"] == 1 and line["value"] > 0 and line["steps"] == 3
    ex = line["exchange"]
    assert ex["chunks"] == 1 and ex["ms_per_step"] > 0 and ex["bytes_per_rank_per_step"] > 0
    want = "reduce" if opts[1] == "reduce" else "sharded+gather"
    assert line["config"]["design"] == want
    names = [v["name"] for v in line["exchange_variants"]]
    assert names[0] == want and len(names) == len(bench_variants())
    assert all(v["value"] > 0 and v["kernel_ms_per_step"] > 0 for v in line["exchange_variants"])
    assert line["roofline"]["kernel"].startswith("k_clients<float, float, 8, 0, 4>")
    # every design (through RCCL at world 1) gives the oracle's round-0 result
    from test_gpu_bench_rehearsal import oracle_check

    want_check = oracle_check(8, 1000003)
    assert line["designs_agree"] is True and line["check"]["decoded_digest"] == want_check
    assert all(v["check_digest"] == want_check for v in line["exchange_variants"])
