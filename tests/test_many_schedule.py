"""Host logic of the pair-shared schedule for more co-located clients than
one fused launch holds (sfl_amd/kernels.py many_schedule / fused_many; GPU
parity in tests/test_gpu_parity.py::test_fused_many_pair_shared_bit_exact)."""
import pytest


@pytest.mark.parametrize("nc", [9, 10, 12, 13, 16, 17, 24, 31, 32, 64, 100])
def test_every_pair_of_clients_exactly_once(nc):
    """Groups (one sa_fused_clients launch each, at most 8 clients) cover the
    pairs inside them, bipartite blocks (two quads in different groups, one
    sa_fused_bipartite launch each) the rest: every pair exactly once, every
    client's quantized value in exactly one group launch, lower quad first."""
    from sfl_amd.kernels import many_schedule

    groups, blocks = many_schedule(nc)
    seen = {}
    assert sorted(c for g in groups for c in g) == list(range(nc))
    for g in groups:
        assert 1 <= len(g) <= 8 and g == sorted(g)
        for i, u in enumerate(g):
            for v in g[i + 1:]:
                seen[(u, v)] = seen.get((u, v), 0) + 1
    for qa, qb in blocks:
        assert 1 <= len(qa) <= 4 and 1 <= len(qb) <= 4 and max(qa) < min(qb)
        for u in qa:
            for v in qb:
                seen[(u, v)] = seen.get((u, v), 0) + 1
    assert len(seen) == nc * (nc - 1) // 2 and set(seen.values()) == {1}
    # draws per element position = the pairs (padding of a short quad aside)
    assert sum(len(g) * (len(g) - 1) // 2 for g in groups) + 16 * len(blocks) >= nc * (nc - 1) // 2
