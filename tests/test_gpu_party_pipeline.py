"""The drop-in's large-payload path: party.mask_payload
and party.sum_decode on host payloads above SMALL_CALL_BYTES run chunked
through three streams (sfl_amd/hostpipe.py: the caller's arrays registered
in place, chunk j's H2D / kernels / D2H overlapping chunk j+1's).  Checked
in-process, as a secretflow PYU would run the functions, against the numpy
oracle: every party's masked vector and XOR digest bit-exact, the stream
positions, the decoded result bit-exact -- over several rounds, layer lists
that straddle chunk joins, every compute type, a non-contiguous and a
read-only input (the registration fallback), a forced raw-0 rejection, and
the per-element-weight / GPU-tensor payloads that keep the one-shot path
(CPU tensors take the pipeline)."""
import dataclasses

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import secagg as o  # noqa: E402

pytestmark = pytest.mark.gpu
NAMES = ["alice", "bob", "carol"]


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd import _lib as L

    L.lib()


def _maskers(seeds):
    from sfl_amd.security.aggregation import party as P

    out = {}
    for nm in NAMES:
        m = P.new_masker(nm)
        out[nm] = P.agree(m, {p: 0 for p in NAMES}, {p: seeds[nm][p] for p in NAMES if p != nm})
    return out


def _expected(layers, w, name, seeds, offset):
    q = np.concatenate([o.quantize(a, None if w is None else (np.broadcast_to(w, np.shape(a)) if np.ndim(w) else w))
                        .reshape(-1) for a in layers])
    return o.mask_client(q, name, seeds[name], offset)


def _payloads(kind, rng):
    """One party's layers for a round kind (sizes well above 1 MiB)."""
    if kind == "f32":
        return [(rng.standard_normal(2_500_003) * 1e-2).astype(np.float32)]
    if kind == "f32_layers":  # several layers, joins inside chunks
        return [(rng.standard_normal((1000, 1500)) * 0.1).astype(np.float32),
                (rng.standard_normal(700_003) * 0.1).astype(np.float32), np.zeros(0, np.float32),
                (rng.standard_normal(1_100_001) * 0.1).astype(np.float32)]
    if kind == "f64":
        return [rng.standard_normal(1_200_007)]
    if kind == "i64":
        return [rng.integers(-1000, 1000, 600_001).astype(np.int64), rng.integers(-9, 9, 700_000).astype(np.int64)]
    if kind == "mixed":  # two launch groups, both large
        return [(rng.standard_normal(1_500_000) * 0.1).astype(np.float32), rng.standard_normal(300_001)]
    if kind == "noncontig":
        return [(rng.standard_normal((2000, 1501)) * 0.1).astype(np.float32).T]
    if kind == "readonly":
        a = (rng.standard_normal(1_300_000) * 0.1).astype(np.float32)
        ro = np.frombuffer(a.tobytes(), dtype=np.float32)
        assert not ro.flags.writeable
        return [ro]
    raise ValueError(kind)


WEIGHTS = {"f32": None, "f32_layers": 0.75, "f64": np.float64(1.5), "i64": 3, "mixed": 2.0,
           "noncontig": None, "readonly": 1.25}


def test_large_payload_rounds_bit_exact():
    from sfl_amd.security.aggregation import party as P

    seeds = o.seeds_for(NAMES)
    maskers = _maskers(seeds)
    rng = np.random.default_rng(5)
    offset = 0
    for kind in ["f32", "f32_layers", "f64", "i64", "mixed", "noncontig", "readonly", "f32"]:
        w = WEIGHTS[kind]
        layers = {nm: _payloads(kind, rng) for nm in NAMES}
        wires = []
        for nm in NAMES:
            payload = layers[nm] if len(layers[nm]) > 1 else layers[nm][0]
            wire, maskers[nm] = P.mask_payload(maskers[nm], payload, w, gpu=0)
            exp = _expected(layers[nm], w, nm, seeds, offset)
            assert wire.u64.dtype == np.uint64 and np.array_equal(wire.u64, exp), (kind, nm)
            assert wire.digest == o.digest(exp), (kind, nm)
            assert wire.positions == {p: offset for p in NAMES if p != nm}
            wires.append(wire)
        n = sum(int(np.prod(np.shape(a))) for a in layers["alice"])
        for average in (False, True):
            got = P.sum_decode(*wires, weights=None if w is None else [w] * 3, average=average, gpu=0)
            flat = np.concatenate([np.asarray(g).reshape(-1) for g in (got if isinstance(got, list) else [got])])
            div = None if not average else (3 if w is None else float(sum([w] * 3)))
            assert np.array_equal(flat, o.decode(o.server_sum([x.u64 for x in wires]), 18, div)), (kind, average)
        offset += n


def test_server_detects_a_changed_large_vector():
    from sfl_amd.security.aggregation import party as P

    seeds = o.seeds_for(NAMES)
    maskers = _maskers(seeds)
    x = (np.random.default_rng(1).standard_normal(1_000_000) * 0.1).astype(np.float32)
    wires = [P.mask_payload(maskers[nm], x, None, gpu=0)[0] for nm in NAMES]
    wires[1].u64[777_777] ^= np.uint64(1)
    with pytest.raises(P.DigestMismatch, match="masked vector 1"):
        P.sum_decode(*wires, gpu=0)


def test_large_payload_rejection_replays_on_numpys_stream():
    """A raw 0 on the (alice, bob) stream at element 1_500_000 of a 2M round:
    the pipelined launch flags it, the device path replays the round from
    the same positions and moves the stream one raw draw further -- numpy's
    Generator.integers rejection (OracleMaskers)."""
    from test_gpu_rejection import forced_zero_state

    from sfl_amd.security.aggregation import party as P

    state = {("alice", "bob"): forced_zero_state(1_500_000)}
    ora = o.OracleMaskers(NAMES[:2], state)
    ms = {}
    for nm in NAMES[:2]:
        m = P.new_masker(nm)
        peer = [p for p in NAMES[:2] if p != nm][0]
        ms[nm] = P.agree(m, {p: 0 for p in NAMES[:2]}, {peer: state[("alice", "bob")]})
    rng = np.random.default_rng(3)
    n = 2_000_000
    for rnd in range(2):
        xs = [(rng.standard_normal(n) * 1e-2).astype(np.float32) for _ in NAMES[:2]]
        wires = []
        for nm, x in zip(NAMES[:2], xs):
            wire, ms[nm] = P.mask_payload(ms[nm], x, None, gpu=0)
            wires.append(wire)
        masked, ssum = ora.round(xs)
        for wire, m in zip(wires, masked):
            assert np.array_equal(wire.u64, m) and wire.digest == o.digest(m), rnd
        assert np.array_equal(P.sum_decode(*wires, gpu=0), o.decode(ssum)), rnd
        assert wires[0].positions == {"bob": rnd * (n + 1)}


def test_per_element_weights_and_device_tensors_keep_the_one_shot_path(monkeypatch):
    from sfl_amd.security.aggregation import party as P

    calls = []
    orig = P._mask_vector_pipelined
    monkeypatch.setattr(P, "_mask_vector_pipelined", lambda *a, **k: calls.append(1) or orig(*a, **k))
    seeds = o.seeds_for(NAMES)
    maskers = _maskers(seeds)
    n = 400_000
    rng = np.random.default_rng(9)
    w = rng.uniform(0.5, 2.0, n)
    x = (rng.standard_normal(n) * 0.1).astype(np.float32)
    wire, _ = P.mask_payload(maskers["alice"], x, w, gpu=0)
    assert np.array_equal(wire.u64, _expected([x], w, "alice", seeds, 0))
    t = torch.from_numpy(x).to("cuda:0")
    wire, _ = P.mask_payload(maskers["alice"], t, None, gpu=0)
    assert np.array_equal(wire.u64, _expected([x], None, "alice", seeds, 0))
    assert calls == []
    # CPU tensors (a state dict's values) are host layers: the pipelined path
    big = (rng.standard_normal(1_500_000) * 0.1).astype(np.float32)
    wire, _ = P.mask_payload(maskers["alice"], [torch.from_numpy(big), torch.from_numpy(x)], None, gpu=0)
    assert calls == [1] and wire.as_torch
    assert np.array_equal(wire.u64, _expected([big, x], None, "alice", seeds, 0))


@pytest.mark.parametrize("C", [2, 5, 8, 12])
def test_in_process_aggregator_large_host_payloads(C, monkeypatch):
    """The in-process SecureAggregator's large host float32 path (co-located
    parties, chunked through three streams like the drop-in) against the
    oracle over two rounds, and against its one-shot path (LARGE_PIPELINE
    off): same results, same per-party digests, same stream positions."""
    from sfl_amd.device import PYU, reveal as rv
    from sfl_amd.security.aggregation import SecureAggregator
    from sfl_amd.security.aggregation import party as P

    names = [f"p{c}" for c in range(C)]
    seeds = o.seeds_for(names)
    pair = {(a, b): seeds[a][b] for a in names for b in names if a != b}
    pyus = [PYU(nm, 0) for nm in names]
    rng = np.random.default_rng(40 + C)
    rounds = [[[(rng.standard_normal((700, 1001)) * 0.1).astype(np.float32),
                (rng.standard_normal(1_300_003) * 0.1).astype(np.float32)] for _ in names] for _ in range(2)]
    weights = [float(w) for w in rng.integers(1, 5, C)]

    def run(pipeline):
        monkeypatch.setattr(P, "LARGE_PIPELINE", pipeline)
        agg = SecureAggregator(PYU("server", 0), pyus, seeds=pair)
        outs = []
        for data in rounds:
            got = rv(agg.average([p(lambda d=d: d)() for p, d in zip(pyus, data)], axis=0, weights=weights))
            outs.append((got, [np.asarray(d).view(np.uint64).copy() for d in agg.last_digests if d is not None]))
        pos = {nm: {q: agg._maskers[nm].position(q) for q in names if q != nm} for nm in names}
        return outs, pos

    a, pos_a = run(True)
    b, pos_b = run(False)
    n = 700 * 1001 + 1_300_003
    assert pos_a == pos_b and all(v == 2 * n for d in pos_a.values() for v in d.values())
    for r, ((ga, da), (gb, db)) in enumerate(zip(a, b)):
        flat = [np.concatenate([x.reshape(-1) for x in d]) for d in rounds[r]]
        exp, _, masked = o.secure_average(flat, names, weights=weights, seeds=seeds, offset=r * n)
        assert [la.shape for la in ga] == [(700, 1001), (1_300_003,)]
        assert np.array_equal(np.concatenate([x.reshape(-1) for x in ga]), exp), r
        assert all(np.array_equal(la, lb) for la, lb in zip(ga, gb)), r
        if C > 8:  # the pair-shared schedule keeps no per-party digests
            assert da == [] and db == []
            continue
        want = [o.digest(m) for m in masked]
        assert [int(x) for x in np.concatenate(da)] == want, r
        assert [int(x) for x in np.concatenate(db)] == want, r


@pytest.mark.parametrize("kind,C", [("f64", 3), ("i64", 3), ("f64", 12)])
def test_in_process_large_general_payloads(kind, C, monkeypatch):
    """float64 / int64 host payloads in process (every party's own sa_mask
    into the sum, chunk by chunk through the three streams) against the
    oracle over two rounds and against the one-shot general path
    (LARGE_PIPELINE off): same results, per-party digests, positions."""
    from sfl_amd.device import PYU, reveal as rv
    from sfl_amd.security.aggregation import SecureAggregator
    from sfl_amd.security.aggregation import party as P
    from sfl_amd.security.aggregation import secure_aggregator as S

    names = [f"p{c}" for c in range(C)]
    seeds = o.seeds_for(names)
    pair = {(a, b): seeds[a][b] for a in names for b in names if a != b}
    pyus = [PYU(nm, 0) for nm in names]
    rng = np.random.default_rng(60 + C)
    if kind == "f64":
        rounds = [[[rng.standard_normal((600, 1001)), rng.standard_normal(700_003)] for _ in names]
                  for _ in range(2)]
        weights = [float(w) for w in rng.uniform(0.5, 3.0, C)]
    else:
        rounds = [[[rng.integers(-1000, 1000, (600, 1001)), rng.integers(-9, 9, 700_003)] for _ in names]
                  for _ in range(2)]
        weights = [int(w) for w in rng.integers(1, 5, C)]
    calls = []
    orig = S.SecureAggregator._host_general_pipelined
    monkeypatch.setattr(S.SecureAggregator, "_host_general_pipelined",
                        lambda *a, **k: calls.append(1) or orig(*a, **k))

    def run(pipeline):
        monkeypatch.setattr(P, "LARGE_PIPELINE", pipeline)
        agg = SecureAggregator(PYU("server", 0), pyus, seeds=pair)
        outs = []
        for data in rounds:
            got = rv(agg.average([p(lambda d=d: d)() for p, d in zip(pyus, data)], axis=0, weights=weights))
            # the one-shot general path keeps its digests on the device
            outs.append((got, [d.cpu().numpy().view(np.uint64).copy() for d in agg.last_digests if d is not None]))
        pos = {nm: {q: agg._maskers[nm].position(q) for q in names if q != nm} for nm in names}
        return outs, pos

    a, pos_a = run(True)
    assert calls == [1, 1]
    b, pos_b = run(False)
    assert calls == [1, 1]
    n = 600 * 1001 + 700_003
    assert pos_a == pos_b and all(v == 2 * n for d in pos_a.values() for v in d.values())
    for r, ((ga, da), (gb, db)) in enumerate(zip(a, b)):
        flat = [np.concatenate([x.reshape(-1) for x in d]) for d in rounds[r]]
        exp, _, masked = o.secure_average(flat, names, weights=weights, seeds=seeds, offset=r * n)
        assert [la.shape for la in ga] == [(600, 1001), (700_003,)]
        assert np.array_equal(np.concatenate([x.reshape(-1) for x in ga]), exp), r
        assert all(np.array_equal(la, lb) for la, lb in zip(ga, gb)), r
        want = [o.digest(m) for m in masked]
        assert [int(x) for x in np.concatenate(da)] == want, r
        assert [int(x) for x in np.concatenate(db)] == want, r


class _NotPinned:
    """H.Pinned stand-in whose registration is refused: the feeder path."""

    def __init__(self, arrays, register=True, lazy=None):
        self.ok = False
        self.spans, self.stats = [], {}

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        return False


@pytest.mark.parametrize("pooled", [True, False])
@pytest.mark.parametrize("pinned", [True, False])
def test_every_copy_path_bit_exact(pooled, pinned, monkeypatch):
    """Each way the pipelined calls move bytes, forced: a party's inputs
    registered (async DMA) or staged through pinned slots by the feeder
    thread; results into recycled registered buffers, or through pinned
    slots into fresh arrays (the drain thread).  Three rounds each (the pool recycles the dropped results
    of the round before), drop-in and in-process, bit-exact vs the oracle."""
    from sfl_amd import hostpipe as H
    from sfl_amd.device import PYU, reveal as rv
    from sfl_amd.security.aggregation import SecureAggregator
    from sfl_amd.security.aggregation import party as P

    monkeypatch.setattr(H, "RESULTS", H.ResultPool((1 << 30) if pooled else 0))
    if not pinned:
        monkeypatch.setattr(H, "Pinned", _NotPinned)
    seeds = o.seeds_for(NAMES)
    maskers = _maskers(seeds)
    rng = np.random.default_rng(77)
    offset = 0
    for rnd in range(3):
        layers = {nm: _payloads("f32_layers" if rnd != 1 else "i64", rng) for nm in NAMES}
        w = 0.75 if rnd != 1 else 3
        wires = []
        for nm in NAMES:
            wire, maskers[nm] = P.mask_payload(maskers[nm], layers[nm], w, gpu=0)
            exp = _expected(layers[nm], w, nm, seeds, offset)
            assert np.array_equal(wire.u64, exp) and wire.digest == o.digest(exp), (rnd, nm)
            wires.append(wire)
        got = P.sum_decode(*wires, weights=[w] * 3, average=True, gpu=0)
        flat = np.concatenate([np.asarray(g).reshape(-1) for g in got])
        assert np.array_equal(flat, o.decode(o.server_sum([x.u64 for x in wires]), 18, float(3 * w))), rnd
        offset += wires[0].u64.size
        del wires, got
    if pooled:
        assert H.RESULTS.bufs, "the pool was used"
    # the in-process aggregator over the same copy paths
    pair = {(a, b): seeds[a][b] for a in NAMES for b in NAMES if a != b}
    pyus = [PYU(nm, 0) for nm in NAMES]
    agg = SecureAggregator(PYU("server", 0), pyus, seeds=pair)
    for rnd in range(2):
        data = [[(rng.standard_normal(1_700_001) * 0.1).astype(np.float32)] for _ in NAMES]
        got = rv(agg.sum([p(lambda d=d: d)() for p, d in zip(pyus, data)], axis=0))
        exp, _, _ = o.secure_sum([d[0] for d in data], NAMES, seeds=seeds, offset=rnd * 1_700_001)
        assert np.array_equal(got[0], exp), rnd
    # int64 layers: the per-party (general) chunked path over the same copy paths
    data = [[rng.integers(-500, 500, 1_300_001)] for _ in NAMES]
    got = rv(agg.sum([p(lambda d=d: d)() for p, d in zip(pyus, data)], axis=0))
    exp, _, _ = o.secure_sum([d[0] for d in data], NAMES, seeds=seeds, offset=2 * 1_700_001)
    assert np.array_equal(got[0], exp)
    del got
    H.RESULTS.clear()


@pytest.mark.parametrize("dtype", [np.float32, np.float64])
def test_in_process_large_rejection_replays_on_numpys_stream(dtype):
    """A raw 0 on the (alice, bob) stream inside the chunked in-process
    launch (element 1_700_000 of a 2.5M round, in a later chunk): the fused
    chunk (float32) or the per-party chunk (float64) flags it, the round is
    replayed in careful mode from the same positions; two rounds equal
    numpy's own generators (OracleMaskers)."""
    from test_gpu_rejection import forced_zero_state

    from sfl_amd.device import PYU, reveal as rv
    from sfl_amd.security.aggregation import SecureAggregator

    names = NAMES
    state = {("alice", "bob"): forced_zero_state(1_700_000)}
    seeds = o.seeds_for(names)
    pairs = {(a, b): state.get((a, b), state.get((b, a), seeds[a][b])) for a in names for b in names if a != b}
    ora = o.OracleMaskers(names, pairs)
    pyus = [PYU(nm, 0) for nm in names]
    agg = SecureAggregator(PYU("server", 0), pyus, seeds=pairs)
    rng = np.random.default_rng(21)
    n = 2_500_000
    for rnd in range(2):
        xs = [(rng.standard_normal(n) * 1e-2).astype(dtype) for _ in names]
        got = rv(agg.sum([p(lambda x=x: x)() for p, x in zip(pyus, xs)], axis=0))
        masked, ssum = ora.round(xs)
        assert np.array_equal(got, o.decode(ssum)), rnd
        dig = agg.last_digests[-1].cpu().numpy().view(np.uint64)
        assert [int(d) for d in dig] == [o.digest(m) for m in masked]
    assert agg._maskers["alice"].position("bob") == 2 * n + 1
    assert agg._maskers["alice"].position("carol") == 2 * n


@pytest.mark.parametrize("growth", [1, 2])
@pytest.mark.parametrize("refuse_after", [None, 2])
def test_lazy_registration_bit_exact(growth, refuse_after, monkeypatch):
    """Inputs registered piece by piece as their copies are issued
    (hostpipe.Pinned lazily: here every array of 1 MiB or more), chunk by
    chunk or doubling, and with the driver refusing every registration after
    the second (the rest of each array staged through pinned temporaries):
    the drop-in's party calls and the in-process float32 / float64 paths
    bit-exact vs the oracle."""
    from sfl_amd import hostpipe as H
    from sfl_amd.device import PYU, reveal as rv
    from sfl_amd.security.aggregation import SecureAggregator
    from sfl_amd.security.aggregation import party as P

    monkeypatch.setattr(H, "LAZY_MIN_BYTES", 1 << 20)
    monkeypatch.setattr(H, "LAZY_GROWTH", growth)
    stats = []
    orig_reg, orig_exit = H.Pinned._reg, H.Pinned.__exit__

    def reg(self, p0, p1):
        if refuse_after is not None and self.stats["registrations"] >= refuse_after:
            return False
        return orig_reg(self, p0, p1)

    def exit_(self, *exc):
        if self.spans:
            stats.append(dict(self.stats))
        return orig_exit(self, *exc)

    monkeypatch.setattr(H.Pinned, "_reg", reg)
    monkeypatch.setattr(H.Pinned, "__exit__", exit_)
    seeds = o.seeds_for(NAMES)
    maskers = _maskers(seeds)
    rng = np.random.default_rng(123)
    layers = {nm: _payloads("f32_layers", rng) for nm in NAMES}
    wires = []
    for nm in NAMES:
        wire, maskers[nm] = P.mask_payload(maskers[nm], layers[nm], 0.75, gpu=0)
        exp = _expected(layers[nm], 0.75, nm, seeds, 0)
        assert np.array_equal(wire.u64, exp) and wire.digest == o.digest(exp), nm
        wires.append(wire)
    want = o.decode(o.server_sum([x.u64 for x in wires]), 18, 2.25)
    got = P.sum_decode(*wires, weights=[0.75] * 3, average=True, gpu=0)
    assert np.array_equal(np.concatenate([np.asarray(g).reshape(-1) for g in got]), want)
    # vectors as another process would hand them over: fresh arrays, not
    # pooled results -- registered lazily by the server, or staged
    for server_register in (True, False):
        monkeypatch.setattr(P, "SERVER_REGISTER", server_register)
        fresh = [dataclasses.replace(w, u64=w.u64.copy()) for w in wires]
        got = P.sum_decode(*fresh, weights=[0.75] * 3, average=True, gpu=0)
        assert np.array_equal(np.concatenate([np.asarray(g).reshape(-1) for g in got]), want), server_register
    pair = {(a, b): seeds[a][b] for a in NAMES for b in NAMES if a != b}
    pyus = [PYU(nm, 0) for nm in NAMES]
    agg = SecureAggregator(PYU("server", 0), pyus, seeds=pair)
    off = 0
    for dt in (np.float32, np.float64):
        data = [[(rng.standard_normal(2_700_001) * 0.1).astype(dt)] for _ in NAMES]
        got = rv(agg.sum([p(lambda d=d: d)() for p, d in zip(pyus, data)], axis=0))
        exp, _, _ = o.secure_sum([d[0] for d in data], NAMES, seeds=seeds, offset=off)
        assert np.array_equal(got[0], exp), dt
        off += 2_700_001
    assert stats and all(s["registrations"] > 0 for s in stats)
    if refuse_after is None:
        assert all(s["staged_bytes"] == 0 for s in stats)
    else:
        assert any(s["staged_bytes"] > 0 for s in stats)


def test_fresh_inputs_at_reused_addresses_bit_exact():
    """Every round's inputs freshly allocated (and the last round's freed),
    as get_weights() hands them over: numpy's large arrays come back at the
    addresses just unmapped, which the driver registered a round before.
    Each round's masked vectors and sum must come from the new pages:
    bit-exact vs the oracle over four rounds of different values, drop-in
    and in-process, with the inputs registered lazily (>= 64 MiB)."""
    from sfl_amd.device import PYU, reveal as rv
    from sfl_amd.security.aggregation import SecureAggregator
    from sfl_amd.security.aggregation import party as P

    n = 17_000_003  # 68 MB of float32 a party
    seeds = o.seeds_for(NAMES)
    maskers = _maskers(seeds)
    pair = {(a, b): seeds[a][b] for a in NAMES for b in NAMES if a != b}
    pyus = [PYU(nm, 0) for nm in NAMES]
    agg = SecureAggregator(PYU("server", 0), pyus, seeds=pair)
    addrs, offset = [], 0
    for rnd in range(4):
        rng = np.random.default_rng(1000 + rnd)
        xs = [(rng.standard_normal(n) * 0.1).astype(np.float32) for _ in NAMES]
        addrs.append(tuple(x.ctypes.data for x in xs))
        wires = []
        for nm, x in zip(NAMES, xs):
            wire, maskers[nm] = P.mask_payload(maskers[nm], x, None, gpu=0)
            exp = _expected([x], None, nm, seeds, offset)
            assert np.array_equal(wire.u64, exp), (rnd, nm)
            wires.append(wire)
        got = rv(agg.sum([p(lambda x=x: x)() for p, x in zip(pyus, xs)], axis=0))
        want, _, _ = o.secure_sum(xs, NAMES, seeds=seeds, offset=offset)
        assert np.array_equal(got, want), rnd
        offset += n
        del xs, wires, got
    print("input addresses per round:", [[hex(a) for a in r] for r in addrs])
