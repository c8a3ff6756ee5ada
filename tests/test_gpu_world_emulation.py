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
