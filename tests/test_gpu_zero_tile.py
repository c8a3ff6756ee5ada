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



# ---------------------------------------------------------------------------
# Every stream of the timed instantiations, at exact element positions
# (VERDICT r4 weak 1 / next 2): the sum-only launches the bench times output
# only the sum, in which every pair mask cancels, so the raw == 0 flag is
# their one mask-dependent observable.  For each stream of each per-rank
# shape, a forced zero at element k must raise the flag with n = k + 1 and
# must NOT with n = k: that pins the stream's jump, increment and slot to
# the exact element (a one-element offset either way fails), at three places
# -- block 0's first tile, a late tile several grid strides on, and past the
# 2^29-element launch-chunk join (kChunkElems, sa_clients_impl.h).
# ---------------------------------------------------------------------------
KCHUNK = (1 << 29) - 512  # kChunkElems: launches are cut into chunks of this many elements
POSITIONS = {"first_tile": 300, "late_tile": 3_000_001, "past_chunk_join": KCHUNK + 1001}
SHAPES = {1: (8, 0), 2: (4, 4), 4: (2, 6), 8: (1, 7)}  # world -> rank 0's (local clients, cross per client)


def forced_zero_state_at(k: int, inc: int = (777 << 1) | 1, tag: int = 0xC0FFEE) -> tuple:
    """(state, inc) whose raw draw k is 0, by one backward jump (k may be
    past 2^29; forced_zero_state steps back one draw at a time)."""
    from test_gpu_rejection import A, M

    ainv = pow(A, -1, 1 << 128)
    s = (((tag << 64) | tag) - inc) * ainv & M  # the state before the zero draw
    s0 = o.pcg64_jump_py(s, inc, (1 << 128) - k)  # k draws further back (the period is 2^128)
    assert o.pcg64_raw_py(o.pcg64_jump_py(s0, inc, k), inc, 1)[0] == 0
    return s0, inc


@pytest.fixture(scope="module")
def big_input():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    n = POSITIONS["past_chunk_join"] + 2
    return torch.randn(n, device=torch.device("cuda", 0)) * 1e-2


@pytest.mark.parametrize("pos", sorted(POSITIONS))
@pytest.mark.parametrize("world", sorted(SHAPES))
def test_every_stream_of_the_timed_shapes_at_exact_positions(world, pos, big_input):
    K, L = _gpu()
    from bench import kernel_variant, pair_seed
    from sfl_amd.parallel_sum import plan_generators, plan_rank

    Lc, X = SHAPES[world]
    names = [f"client{c}" for c in range(8)]
    plan = plan_rank(names, world, 0)
    assert (len(plan.clients), len(plan.cross) // max(1, len(plan.clients))) == (Lc, X)
    assert kernel_variant(Lc, X, False) in (4, 6)  # the sum-only instantiation the bench times
    pg0, ps, cross0 = plan_generators(plan, pair_seed)
    k = POSITIONS[pos]
    zero = L.PCG64.of(*forced_zero_state_at(k))
    dev = big_input.device
    s = torch.empty(k + 1, dtype=torch.int64, device=dev)
    flags = torch.zeros(1, dtype=torch.int32, device=dev)
    missed = []
    for j in range(len(pg0) + len(cross0)):
        pg, cross = list(pg0), list(cross0)
        if j < len(pg):
            pg[j] = zero
        else:
            g, sign, peer = cross[j - len(pg)]
            cross[j - len(pg)] = (zero, sign, peer)
        for n, want in ((k + 1, True), (k, False)):
            flags.zero_()
            xs = [big_input[:n]] * Lc  # the clients' values do not enter the flag
            K.fused_clients(xs, [1.0] * Lc, pg, ps, cross, X, s[:n], flags=flags)
            torch.cuda.synchronize()
            got = bool(int(flags.item()) & L.SA_FLAG_PRG_REJECT)
            if got != want:
                missed.append((j, n, got))
    assert not missed, f"world {world} (<{Lc},{X}>) zero at element {k}: (stream, n, flag) wrong: {missed}"


def _flag_matrix(K, L, launch, n_streams, k):
    """For each stream j: forced zero at element k; flag expected with
    n = k + 1, none with n = k.  ``launch(j, zero, n, flags)`` runs the
    launch set with stream j replaced.  Returns the wrong (j, n, flag)."""
    zero = L.PCG64.of(*forced_zero_state_at(k))
    dev = torch.device("cuda", 0)
    flags = torch.zeros(1, dtype=torch.int32, device=dev)
    missed = []
    for j in range(n_streams):
        for n, want in ((k + 1, True), (k, False)):
            flags.zero_()
            launch(j, zero, n, flags)
            torch.cuda.synchronize()
            got = bool(int(flags.item()) & L.SA_FLAG_PRG_REJECT)
            if got != want:
                missed.append((j, n, got))
    return missed


@pytest.mark.parametrize("pos", sorted(POSITIONS))
def test_config5_rank_schedule_every_stream_at_exact_positions(pos, big_input):
    """Config 5 at 8 GPUs, rank 0: 4 local clients, 6 internal pairs and 4 x
    28 cross streams -- the multi-launch schedule the bench times (a fused
    <4,4,4> launch, then 3 masks-only <1,32,14> launches adding into the sum).
    Every one of the 118 streams (past the chunk join: every 5th) at the
    exact element."""
    K, L = _gpu()
    from bench import pair_seed
    from sfl_amd.parallel_sum import plan_generators, plan_rank

    names = [f"client{c}" for c in range(32)]
    plan = plan_rank(names, 8, 0)
    Lc, X = len(plan.clients), len(plan.cross) // len(plan.clients)
    assert (Lc, X) == (4, 28)
    pg0, ps, cross0 = plan_generators(plan, pair_seed)
    k = POSITIONS[pos]
    s = torch.empty(k + 1, dtype=torch.int64, device=big_input.device)
    streams = list(range(len(pg0) + len(cross0)))
    if pos == "past_chunk_join":
        streams = streams[::5] + [streams[-1]]

    def launch(j, zero, n, flags):
        pg, cross = list(pg0), list(cross0)
        jj = streams[j]
        if jj < len(pg):
            pg[jj] = zero
        else:
            g, sign, peer = cross[jj - len(pg)]
            cross[jj - len(pg)] = (zero, sign, peer)
        K.fused_clients([big_input[:n]] * Lc, [1.0] * Lc, pg, ps, cross, X, s[:n], flags=flags)

    missed = _flag_matrix(K, L, launch, len(streams), k)
    assert not missed, f"config-5 rank schedule, zero at element {k}: (stream, n, flag) wrong: {missed}"


@pytest.mark.parametrize("pos", sorted(POSITIONS))
def test_bipartite_block_every_stream_at_exact_positions(pos, big_input):
    """The masks-only sa_fused_bipartite launch (k_clients<8,0,1>: the 16 pairs
    between two quads of co-located clients; config 5 on one GPU runs 24 of
    them per step): each of its 16 streams at the exact element."""
    import ctypes as C

    K, L = _gpu()
    names = [f"client{c}" for c in range(8)]
    seeds = o.seeds_for(names)
    gens0 = [L.pcg64_from_seed(seeds[names[i]][names[4 + j]]) for i in range(4) for j in range(4)]
    signs = (C.c_int8 * 16)(*[1 if (i + j) % 2 else -1 for i in range(4) for j in range(4)])
    clients = (L.LocalClient * 8)()
    for c in range(8):
        clients[c].x, clients[c].weight, clients[c].masked_out = None, 1.0, None
    k = POSITIONS[pos]
    s = torch.zeros(k + 1, dtype=torch.int64, device=big_input.device)

    def launch(j, zero, n, flags):
        gens = list(gens0)
        gens[j] = zero
        L.check(L.lib().sa_fused_bipartite(clients, L.SA_F32, n, 18, (L.PCG64 * 16)(*gens), signs,
                                           C.c_void_p(s.data_ptr()), 1, C.c_void_p(flags.data_ptr()),
                                           C.c_void_p(torch.cuda.current_stream().cuda_stream)),
                "sa_fused_bipartite")

    missed = _flag_matrix(K, L, launch, 16, k)
    assert not missed, f"bipartite block, zero at element {k}: (stream, n, flag) wrong: {missed}"
