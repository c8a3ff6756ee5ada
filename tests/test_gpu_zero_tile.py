"""The masking kernel's raw == 0 test (numpy's Lemire draw re-draws a raw 0)
in a LATE tile of a wave: the paired draws (sa_draw2.h) and the single draws
(SA_PCG_DRAW_ASM) OR their compare masks into per-tile SGPR masks that the
tile folds into the lane's running minimum, so a zero in any tile of any
wave must reach SA_FLAG_PRG_REJECT.  Vectors longer than one grid stride of
tiles put the forced zero in a wave's third tile; a control launch with the
same shape and no zero leaves the flag clear."""
import pytest

from oracle import secagg as o
from test_gpu_rejection import forced_zero_state

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu


def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd import _lib as L
    from sfl_amd import kernels as K

    return K, L


def _launch(K, L, n, L_clients, gens, signs, cross, n_cross):
    dev = torch.device("cuda", 0)
    xs = [torch.randn(n, device=dev) * 1e-2 for _ in range(L_clients)]
    s = torch.empty(n, dtype=torch.int64, device=dev)
    flags = torch.zeros(1, dtype=torch.int32, device=dev)
    K.fused_clients(xs, [1.0] * L_clients, gens, signs, cross, n_cross, s, flags=flags)
    torch.cuda.synchronize()
    return int(flags.item())


@pytest.mark.parametrize("zero_pair", [None, 0, 27])
def test_eight_clients_zero_in_late_tile(zero_pair):
    """8 co-located clients (28 pair streams, all in paired draw blocks): a
    zero drawn by pair stream `zero_pair` at element 600,001 -- beyond two
    grid strides of 512-element tiles -- sets the flag."""
    K, L = _gpu()
    n, k = 700_003, 600_001
    names = [f"client{c}" for c in range(8)]
    seeds = o.seeds_for(names)
    gens, signs = [], []
    for u in range(8):
        for v in range(u + 1, 8):
            gens.append(L.pcg64_from_seed(seeds[names[u]][names[v]]))
            signs.append(1)
    if zero_pair is not None:
        gens[zero_pair] = L.PCG64.of(*forced_zero_state(k))
    f = _launch(K, L, n, 8, gens, signs, [], 0)
    assert bool(f & L.SA_FLAG_PRG_REJECT) == (zero_pair is not None), f


@pytest.mark.parametrize("zero_stream", [None, 0, 2])
def test_one_client_three_cross_streams_zero_in_late_tile(zero_stream):
    """One client with 3 cross streams: streams 0 and 1 share a paired block,
    stream 2 is a single draw; a zero at element 2,300,001 (past the lean
    kernel's larger grid stride twice) in either kind sets the flag."""
    K, L = _gpu()
    n, k = 2_400_007, 2_300_001
    seeds = o.seeds_for(["a", "b", "c", "d"])
    cross = []
    for j, p in enumerate(["b", "c", "d"]):
        g = L.pcg64_from_seed(seeds["a"][p])
        if zero_stream == j:
            g = L.PCG64.of(*forced_zero_state(k))
        cross.append((g, 1, j))
    f = _launch(K, L, n, 1, [], [], cross, 3)
    assert bool(f & L.SA_FLAG_PRG_REJECT) == (zero_stream is not None), f

