"""sa_fused_clients' multi-launch schedule: per-rank shapes with more streams
than one launch holds, only the masked sum wanted (config 5 at 8 GPUs: 32
clients, 4 per GPU -> 6 internal pairs + 4 x 28 cross streams = 118 streams
per element position).  The schedule draws every internal pair ONCE: a fused
sum-only launch with the pairs and the first cross streams of every client,
then masks-only launches (k_clients<1, X, kLean1|kSumOnly|kCrossOnly>) of
the remaining cross streams adding into the sum -- instead of the per-client
fallback's two sa_mask passes per client (124 draws + masked-vector round
trips).  Every result is compared with the oracle (reference equation:
docs/developer/algorithm/secure_aggregation.ipynb:229)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


def _rank_oracle(xs, names, seeds, plan, n, offset):
    from oracle import secagg as o

    exp = np.zeros(n, dtype=np.uint64)
    for c in plan.clients:
        exp += o.mask_client(o.quantize(xs[c]), names[c], seeds[names[c]], offset)
    return exp


# (C, W, ranks): 4+28 (config 5 at 8 GPUs), 8+24 (config 5 at 4 GPUs), 5+35,
# 4+32, and single clients with 34 / 41 cross streams (remainders that take
# the 24/16/8/4/2/1-stream masks-only kernels)
SHAPES = [(32, 8, range(8)), (32, 4, (0, 3)), (40, 8, (2,)), (36, 9, (4,)), (35, 35, (5,)), (42, 42, (0,))]


@pytest.mark.parametrize("C,W,ranks", SHAPES)
@pytest.mark.parametrize("accumulate", [False, True])
def test_multi_launch_schedule_vs_oracle(C, W, ranks, accumulate):
    from oracle import secagg as o
    from sfl_amd import kernels as K
    from sfl_amd.parallel_sum import plan_generators, plan_rank

    n, offset = 5003, 7 + C
    names = [f"c{i:02d}" for i in range(C)]
    seeds = o.seeds_for(names)
    seed_of = lambda u, v: seeds[names[u]][names[v]]  # noqa: E731
    rng = np.random.default_rng(C * 100 + W)
    xs = [(rng.standard_normal(n) * 1e-2).astype(np.float32) for _ in range(C)]
    for r in ranks:
        plan = plan_rank(names, W, r)
        assert len(plan.pairs) + len(plan.cross) > 32  # beyond one launch
        pg, ps, cross = plan_generators(plan, seed_of, offset=offset)
        init = rng.integers(0, 2**63, n, dtype=np.int64)
        s = torch.from_numpy(init).to(DEV) if accumulate else torch.empty(n, dtype=torch.int64, device=DEV)
        flags = torch.zeros(1, dtype=torch.int32, device=DEV)
        K.fused_clients([torch.from_numpy(xs[c]).to(DEV) for c in plan.clients], [1.0] * len(plan.clients), pg, ps,
                        cross, plan.n_cross, s, accumulate=accumulate, flags=flags)
        torch.cuda.synchronize()
        exp = _rank_oracle(xs, names, seeds, plan, n, offset)
        if accumulate:
            exp += init.view(np.uint64)
        assert np.array_equal(K.as_u64(s), exp), (C, W, r)
        assert int(flags.item()) == 0


def test_multi_launch_equals_per_client_fallback_and_flags_a_zero_draw():
    """The schedule's sum equals the per-client path's (digests requested ->
    sa_mask passes) at 1M elements on every rank of 32 clients over 8 GPUs,
    and a raw PCG64 draw of 0 in a cross stream of a LATER (masks-only)
    launch raises the rejection flag like the first launch does."""
    from oracle import secagg as o
    from sfl_amd import _lib as L
    from sfl_amd import kernels as K
    from sfl_amd.parallel_sum import plan_generators, plan_rank
    from test_gpu_rejection import forced_zero_state

    C, W, n = 32, 8, 1_000_003
    names = [f"client{c}" for c in range(C)]
    seeds = o.seeds_for(names)
    seed_of = lambda u, v: seeds[names[u]][names[v]]  # noqa: E731
    for r in range(W):
        plan = plan_rank(names, W, r)
        Lc = len(plan.clients)
        xs = [torch.randn(n, device=DEV) * 1e-2 for _ in range(Lc)]
        pg, ps, cross = plan_generators(plan, seed_of, offset=11 * n)
        s = torch.empty(n, dtype=torch.int64, device=DEV)
        K.fused_clients(xs, [1.0] * Lc, pg, ps, cross, plan.n_cross, s)
        s_ref = torch.empty(n, dtype=torch.int64, device=DEV)
        dig = torch.zeros(Lc, dtype=torch.int64, device=DEV)
        K.fused_clients(xs, [1.0] * Lc, pg, ps, cross, plan.n_cross, s_ref, digests=dig)  # per-client path
        torch.cuda.synchronize()
        assert torch.equal(s, s_ref), r
    # the last client's last cross stream is drawn by the last masks-only launch
    bad = list(cross)
    bad[-1] = (L.PCG64.of(*forced_zero_state(777)), bad[-1][1], bad[-1][2])
    flags = torch.zeros(1, dtype=torch.int32, device=DEV)
    K.fused_clients(xs, [1.0] * Lc, pg, ps, bad, plan.n_cross, s, flags=flags)
    torch.cuda.synchronize()
    assert int(flags.item()) & L.SA_FLAG_PRG_REJECT


def test_config5_per_rank_schedule_full_size():
    """Config 5's per-rank shape at its full size (32 clients x 256M, 4 per
    GPU over 8 GPUs), run as bench.py runs it (8-chunk pipeline, streams a
    round in), for every rank: the ranks' partial sums add up to the plain
    quantized sum (the masks cancel across ranks), and each rank's launches
    equal the oracle on windows of 4096 at both ends, the middle, across
    every chunk join and at random offsets."""
    from oracle import secagg as o
    from oracle_windows import check_partial_sum_windows
    from sfl_amd import kernels as K
    from sfl_amd.parallel_sum import PipelinedMaskedSum, plan_generators, plan_rank

    C, W, n, offset = 32, 8, 256_000_000, 256_000_000 + 5
    names = [f"client{c}" for c in range(C)]
    seeds = o.seeds_for(names)
    seed_of = lambda u, v: seeds[names[u]][names[v]]  # noqa: E731
    dev = torch.device(DEV)
    xs = []
    for c in range(C):
        g = torch.Generator(device=dev).manual_seed(3100 + c)
        xs.append(torch.randn(n, generator=g, device=dev, dtype=torch.float32) * 1e-2)
    q_sum = torch.zeros(n, dtype=torch.int64, device=dev)
    qbuf = torch.empty(n, dtype=torch.int64, device=dev)
    for x in xs:
        K.mask(x, qbuf, [], sum_accum=q_sum)
    del qbuf
    total = torch.zeros(n, dtype=torch.int64, device=dev)
    part = torch.empty(n, dtype=torch.int64, device=dev)
    pipe = PipelinedMaskedSum(None, dev, n, 8)
    joins = [lo for lo, _ in pipe.bounds[1:]]
    for r in range(W):
        plan = plan_rank(names, W, r)
        gens = [plan_generators(plan, seed_of, offset=offset + lo) for lo, _ in pipe.bounds]
        flags = torch.zeros(1, dtype=torch.int32, device=dev)
        pipe.run([xs[c] for c in plan.clients], [1.0] * len(plan.clients), gens, plan.n_cross, part, None,
                 flags=flags)
        total += part
        torch.cuda.synchronize()
        assert int(flags.item()) == 0
        assert check_partial_sum_windows(part, xs, plan.clients, names, seeds, offset, joins=joins, k_random=3,
                                         seed=r) >= 8 * 4096
    torch.cuda.synchronize()
    assert torch.equal(total, q_sum)


def test_masking_reserve_leaves_results_unchanged():
    """sa_set_masking_reserve (CUs of the masking grid left free for the
    overlapped exchange) changes only which tiles a block takes: the sum of a
    fused launch, of the multi-launch schedule and of a single-client pass is
    bit-identical at every reserve; out-of-range values are refused."""
    from oracle import secagg as o
    from sfl_amd import _lib as L
    from sfl_amd import kernels as K
    from sfl_amd.parallel_sum import plan_generators, plan_rank

    n = 3_000_017
    names = [f"client{c}" for c in range(32)]
    seeds = o.seeds_for(names)
    seed_of = lambda u, v: seeds[names[u]][names[v]]  # noqa: E731
    outs = []
    try:
        for r in (0, 8, 64, 128):
            L.check(L.lib().sa_set_masking_reserve(r), "reserve")
            res = []
            for W in (8, 4, 32):  # 4 + 28 (multi-launch), 8 + 24 (multi-launch), 1 + 31 (passes)
                plan = plan_rank(names, W, 1)
                torch.manual_seed(W)
                xs = [torch.randn(n, device=DEV) * 1e-2 for _ in plan.clients]
                pg, ps, cross = plan_generators(plan, seed_of, offset=5)
                s = torch.empty(n, dtype=torch.int64, device=DEV)
                K.fused_clients(xs, [1.0] * len(xs), pg, ps, cross, plan.n_cross, s)
                res.append(s)
            torch.cuda.synchronize()
            outs.append(res)
    finally:
        L.lib().sa_set_masking_reserve(0)
    for res in outs[1:]:
        for a, b in zip(outs[0], res):
            assert torch.equal(a, b)
    assert L.lib().sa_set_masking_reserve(-1) != L.SA_OK and L.lib().sa_set_masking_reserve(129) != L.SA_OK
