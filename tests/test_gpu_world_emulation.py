"""Every rank of the multi-GPU layout, run one after another on one MI355X.

The driver's N = 2, 4, 8 bench runs one process per GPU; rank r launches
the fused kernel for its block of clients (``plan_rank``: L = 8/W local
clients, 8 - L cross streams each, shapes k_clients<4,4>, <2,6>, <1,7>)
through the same ``PipelinedMaskedSum`` chunking bench.py uses, then RCCL
reduces the uint64 partial sums.  Here each rank's launches run with no
communicator and the partial sums are added on the device (int64 addition
wraps like uint64, the reduce's arithmetic): the total must equal the
oracle's server sum bit for bit, and every client's digest the oracle's.
"""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("W", [1, 2, 4, 8])
@pytest.mark.parametrize("chunks", [1, 8])
def test_all_ranks_sum_to_the_oracle(W, chunks):
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import secagg as o
    from sfl_amd.parallel_sum import PipelinedMaskedSum, plan_generators, plan_rank

    C, n, offset = 8, 70_001, 3 * 10**9 + 17  # a later round: streams start far in
    names = [f"client{c}" for c in range(C)]
    seeds = o.seeds_for(names)
    rng = np.random.default_rng(100 * W + chunks)
    xs = [(rng.standard_normal(n) * 1e-2).astype(np.float32) for _ in range(C)]
    masked = o.secure_masked(xs, names, seeds=seeds, offset=offset)
    exp = o.server_sum(masked)

    dev = torch.device("cuda", 0)
    seed_of = lambda u, v: seeds[names[u]][names[v]]  # noqa: E731
    total = torch.zeros(n, dtype=torch.int64, device=dev)
    digests = {}
    for r in range(W):
        plan = plan_rank(names, W, r)
        assert len(plan.clients) == C // W and plan.n_cross == C - C // W
        pipe = PipelinedMaskedSum(None, dev, n, chunks)
        gens = [plan_generators(plan, seed_of, offset=offset + lo) for lo, _ in pipe.bounds]
        part = torch.empty(n, dtype=torch.int64, device=dev)
        dig = torch.zeros(len(plan.clients), dtype=torch.int64, device=dev)
        flags = torch.zeros(1, dtype=torch.int32, device=dev)
        pipe.run([torch.from_numpy(xs[c]).to(dev) for c in plan.clients], [1.0] * len(plan.clients), gens,
                 plan.n_cross, part, None, digests=dig, flags=flags)
        total += part
        torch.cuda.synchronize()
        assert int(flags.item()) == 0
        for c, d in zip(plan.clients, dig.cpu().numpy().view(np.uint64)):
            digests[c] = int(d)
    assert np.array_equal(total.cpu().numpy().view(np.uint64), exp)
    assert [digests[c] for c in range(C)] == [o.digest(m) for m in masked]
    # the masks cancel: the decoded total is the plain quantized sum
    assert np.array_equal(exp, o.server_sum([o.quantize(x) for x in xs]))


@pytest.mark.parametrize("W", [2, 4, 8])
def test_per_rank_shapes_full_size(W):
    """Every per-rank shape of the N = 2, 4, 8 bench (k_clients<4,4>, <2,6>,
    <1,7>) at the headline size, 100M element positions, run as bench.py
    runs it (8-chunk pipeline, streams a round in) for every rank:

    1. the ranks' partial sums add up to the plain quantized sum (the masks
       cancel across ranks);
    2. each rank's pipelined fused partial sum and digests equal the wire
       path's: every local client masked by its own sa_mask launch (all 7 of
       its streams), summed with sa_sum_u64;
    3. one unchunked fused launch with wire images per rank equals those
       per-client vectors bit for bit, and oracle spot checks (numpy
       Generator at far stream offsets) pin individual elements, including
       both ends and elements either side of the pipeline's chunk joins."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import secagg as o
    from oracle_windows import check_partial_sum_windows
    from sfl_amd import _lib as L
    from sfl_amd import kernels as K
    from sfl_amd.parallel_sum import PipelinedMaskedSum, plan_generators, plan_rank

    C, n, offset = 8, 100_000_000, 5 * 10**9 + 3
    names = [f"client{c}" for c in range(C)]
    seeds = o.seeds_for(names)
    seed_of = lambda u, v: seeds[names[u]][names[v]]  # noqa: E731
    dev = torch.device("cuda", 0)
    xs = []
    for c in range(C):
        g = torch.Generator(device=dev).manual_seed(900 + c)
        xs.append(torch.randn(n, generator=g, device=dev, dtype=torch.float32) * 1e-2)
    q_sum = torch.zeros(n, dtype=torch.int64, device=dev)
    qbuf = torch.empty(n, dtype=torch.int64, device=dev)
    for x in xs:
        K.mask(x, qbuf, [], sum_accum=q_sum)
    del qbuf
    total = torch.zeros(n, dtype=torch.int64, device=dev)
    rng = np.random.default_rng(W)
    pipe = PipelinedMaskedSum(None, dev, n, 8)
    joins = [lo for lo, _ in pipe.bounds[1:]]
    idx = np.unique(np.concatenate([[0, 1, n - 2, n - 1], [j - 1 for j in joins], joins, rng.integers(0, n, 12)]))
    for r in range(W):
        plan = plan_rank(names, W, r)
        Lc = len(plan.clients)
        local = [xs[c] for c in plan.clients]
        # (1)+(2) the bench's pipelined launches
        gens = [plan_generators(plan, seed_of, offset=offset + lo) for lo, _ in pipe.bounds]
        part = torch.empty(n, dtype=torch.int64, device=dev)
        dig = torch.zeros(Lc, dtype=torch.int64, device=dev)
        flags = torch.zeros(1, dtype=torch.int32, device=dev)
        pipe.run(local, [1.0] * Lc, gens, plan.n_cross, part, None, digests=dig, flags=flags)
        total += part
        # as bench.py launches it: no digests (the kernel's sum-only finish)
        part_so = torch.empty(n, dtype=torch.int64, device=dev)
        pipe.run(local, [1.0] * Lc, gens, plan.n_cross, part_so, None)
        torch.cuda.synchronize()
        assert torch.equal(part_so, part), r
        # the bench's launches themselves pinned to the oracle: windows of
        # 4096 at both ends, the middle, across every chunk join and at
        # random offsets (the <1,7> lean shape at W = 8)
        assert check_partial_sum_windows(part_so, xs, plan.clients, names, seeds, offset, joins=joins,
                                         seed=r) >= 8 * 4096
        del part_so
        wire, wdig = [], torch.zeros(Lc, dtype=torch.int64, device=dev)
        for i, c in enumerate(plan.clients):
            st = [(L.pcg64_advance(L.pcg64_from_seed(seed_of(c, v)), offset), 1 if names[v] > names[c] else -1, v)
                  for v in range(C) if v != c]
            out = torch.empty(n, dtype=torch.int64, device=dev)
            K.mask(xs[c], out, st, digest=wdig[i:i + 1])
            wire.append(out)
        wsum = K.sum_u64(wire, torch.empty(n, dtype=torch.int64, device=dev))
        torch.cuda.synchronize()
        assert int(flags.item()) == 0
        assert torch.equal(part, wsum), r
        assert torch.equal(dig, wdig), r
        del wsum
        # (3) one unchunked fused launch storing the wire images
        pg, ps, cross = plan_generators(plan, seed_of, offset=offset)
        imgs = [torch.empty(n, dtype=torch.int64, device=dev) for _ in plan.clients]
        s1 = torch.empty(n, dtype=torch.int64, device=dev)
        K.fused_clients(local, [1.0] * Lc, pg, ps, cross, plan.n_cross, s1, masked_outs=imgs)
        torch.cuda.synchronize()
        assert torch.equal(s1, part), r
        for i, c in enumerate(plan.clients):
            assert torch.equal(imgs[i], wire[i]), (r, c)
            got = imgs[i][torch.from_numpy(idx).to(dev)].cpu().numpy().view(np.uint64)
            xh = xs[c][torch.from_numpy(idx).to(dev)].cpu().numpy()
            for t, e in enumerate(idx):
                v = int(o.quantize(xh[t:t + 1])[0])
                for p in names:
                    if p != names[c]:
                        m = int(o.mask_stream(seeds[names[c]][p], 1, offset + int(e))[0])
                        v = (v + m) & o.U64 if p > names[c] else (v - m) & o.U64
                assert int(got[t]) == v, (r, c, int(e))
        del wire, imgs, s1, part
    torch.cuda.synchronize()
    assert torch.equal(total, q_sum)


@pytest.mark.parametrize("world", [2, 8])
def test_element_sharding_slices_match_oracle(world):
    """bench.py --shard elements: every rank masks its slice of ALL 8 clients
    in one fused launch with the pair streams jumped to the slice start; the
    ranks' slices of the masked sum (and of its decode) laid side by side
    equal the oracle's whole-vector sum, in round 3 of a run (stream
    positions 3n + e0)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import secagg as o
    from sfl_amd import kernels as K
    from sfl_amd.parallel_sum import element_shard, plan_generators, plan_rank

    C, n, rnd = 8, 90_011, 3
    names = [f"client{c}" for c in range(C)]
    seeds = o.seeds_for(names)
    seed_of = lambda u, v: seeds[names[u]][names[v]]  # noqa: E731
    rng = np.random.default_rng(world)
    xs = [(rng.standard_normal(n) * 1e-2).astype(np.float32) for _ in range(C)]
    ssum = o.server_sum(o.secure_masked(xs, names, seeds=seeds, offset=rnd * n))
    plan = plan_rank(names, 1, 0)
    dev = torch.device("cuda", 0)
    got_s, got_d = [], []
    for r in range(world):
        e0, m, k = element_shard(n, world, r)
        pg, ps, cross = plan_generators(plan, seed_of, offset=rnd * n + e0)
        s = torch.zeros(k, dtype=torch.int64, device=dev)
        K.fused_clients([torch.from_numpy(x[e0:e0 + m].copy()).to(dev) for x in xs], [1.0] * C, pg, ps, cross, 0,
                        s[:m])
        d = K.decode(s, torch.empty(k, dtype=torch.float64, device=dev))
        torch.cuda.synchronize()
        got_s.append(s[:m].cpu().numpy().view(np.uint64))
        got_d.append(d[:m].cpu().numpy())
    assert np.array_equal(np.concatenate(got_s), ssum)
    assert np.array_equal(np.concatenate(got_d), o.decode(ssum))
