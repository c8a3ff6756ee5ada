"""The secretflow drop-in (sfl_amd.compat.secretflow) against a secretflow
stand-in with real party isolation (tests/fake_secretflow.py): every party is
a spawned process, the driver holds opaque handles, and ``reveal`` raises on
any client-owned value but a public key.

What is checked, per the reference's protocol
(docs/developer/algorithm/secure_aggregation.ipynb:227-258;
sfl/security/aggregation/sparse_plain_aggregator.py:86,96;
stateful_fedgen_aggregator.py:20-33,74-85):

* each participant's masker is created by -- and stays in -- its own process;
  the driver reveals the DH public keys and nothing else of a client, and
  holds no Masker / DiffieHellman object;
* the masked vector each client sends equals the oracle's (explicit seeds),
  round after round (stream positions persist inside the parties);
* the 7 AggregatorBase cases (tests/security/aggregation/test_aggregator_base.py:21-160)
  come out bit-exact vs the oracle, with device-object weights used on their
  own party;
* ``install()`` rebinds secretflow.security AND .aggregation; a subclass
  defined after it (the reference's StatefulFedGenAggregator pattern)
  aggregates through the drop-in; one defined before makes install() raise.

CPU: the party processes run the oracle's arithmetic in place of the two
device steps (tests/party_oracle_backend.py); GPU: the HIP steps
(``sa_mask`` in each client process, ``sa_sum_u64`` + ``sa_decode`` in the
server's)."""
import gc
import importlib.util
import json
import os

import numpy as np
import pytest

torch = pytest.importorskip("torch")

import fake_secretflow as fs  # noqa: E402
from oracle import secagg as o  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
CONTRACT = json.load(open(os.path.join(HERE, "golden", "aggregator_contract.json")))
NAMES = ["alice", "bob"]
REF_SUBCLASS = "/root/reference/sfl/security/aggregation/stateful_fedgen_aggregator.py"


def _oracle_backend_init():
    import party_oracle_backend

    party_oracle_backend.install()


def _cluster(oracle_backend: bool):
    init = _oracle_backend_init if oracle_backend else None
    return fs.Cluster(NAMES + ["carol"], private=NAMES, init=init)


@pytest.fixture(scope="module")
def cpu_cluster():
    c = _cluster(True)
    yield c
    c.close()


def _seeds():
    s = o.seeds_for(NAMES)
    return s, {(a, b): s[a][b] for a in NAMES for b in NAMES if a != b}


def _put(dev, value):
    return dev(lambda v: v)(value)


def _case_inputs(case):
    a, b = case["a"], case["b"]
    if isinstance(a[0][0], list):  # a list of layers
        return [np.array(x) for x in a], [np.array(x) for x in b]
    return np.array(a), np.array(b)


def _flat(v):
    return np.concatenate([np.asarray(x, dtype=np.float64).reshape(-1) for x in v]) if isinstance(v, (list, tuple)) \
        else np.asarray(v, dtype=np.float64).reshape(-1)


def _cat(v):
    """Layers packed in order, element type kept (the oracle quantizes by it)."""
    return np.concatenate([np.asarray(x).reshape(-1) for x in v]) if isinstance(v, list) else np.asarray(v).reshape(-1)


def _run_contract(cluster, agg, seeds, weights_on_device: bool):
    """The 7 AggregatorBase cases in order on one aggregator; the stream
    positions advance by each case's element count."""
    alice, bob, carol = (cluster.pyu(n) for n in NAMES + ["carol"])
    offset = 0
    for name in ("sum_single", "sum_list", "avg_single", "avg_list", "avg_weights", "avg_list_weights",
                 "avg_same_shape_weights"):
        case = CONTRACT[name]
        xa, xb = _case_inputs(case)
        da, db = _put(alice, xa), _put(bob, xb)
        w = None
        if "weights" in case:
            w = np.array(case["weights"]) if name == "avg_same_shape_weights" else list(case["weights"])
        if name.startswith("sum"):
            out = agg.sum([da, db], axis=0)
        elif w is not None and weights_on_device and name != "avg_same_shape_weights":
            out = agg.average([da, db], axis=0, weights=[_put(alice, w[0]), _put(bob, w[1])])
        else:
            out = agg.average([da, db], axis=0, weights=w)
        assert out.device == carol
        got = fs.reveal(out)  # server-owned: revealable
        # oracle, same seeds and stream positions
        xs = [_cat(xa), _cat(xb)]
        if name.startswith("sum"):
            exp, _, masked = o.secure_sum(xs, NAMES, seeds=seeds, offset=offset)
        else:
            ow = None
            if w is not None:
                ow = [np.broadcast_to(w[0], np.shape(xa)).reshape(-1), np.broadcast_to(w[1], np.shape(xb)).reshape(-1)] \
                    if name == "avg_same_shape_weights" else w
            exp, _, masked = o.secure_average(xs, NAMES, weights=ow, seeds=seeds, offset=offset)
        assert np.array_equal(_flat(got), exp), name
        # what the server received is each client's masked vector, bit for bit
        recv = [fs.reveal(m) for m in agg.last_masked]
        for r, m in zip(recv, masked):
            assert np.array_equal(r.u64, np.asarray(m, dtype=np.uint64).reshape(-1)), name
        # and the reference's contract values
        expect = case.get("expect")
        if expect is None:
            expect = np.average([np.array(case["a"]), np.array(case["b"])], axis=0, weights=np.array(case["weights"]))
        if isinstance(got, list):
            for g, e in zip(got, expect):
                np.testing.assert_almost_equal(g, np.array(e), decimal=case["decimal"])
        else:
            np.testing.assert_almost_equal(got, np.array(expect), decimal=case["decimal"])
        offset += xs[0].size


def _driver_holds(*names):
    return [type(x).__name__ for x in gc.get_objects() if type(x).__name__ in names]


def test_masking_stays_inside_each_party(cpu_cluster):
    from sfl_amd.compat import secretflow as hip

    c = cpu_cluster
    seeds, pair = _seeds()
    c.reveals.clear()
    agg = hip.SecureAggregator(c.pyu("carol"), [c.pyu(n) for n in NAMES], reveal=fs.reveal, seeds=pair)
    # set-up revealed exactly the two public keys
    assert c.reveals == [("alice", "int"), ("bob", "int")]
    _run_contract(c, agg, seeds, weights_on_device=True)
    assert c.reveals[:2] == [("alice", "int"), ("bob", "int")]
    assert all(p == "carol" for p, _ in c.reveals[2:]), c.reveals
    assert _driver_holds("Masker", "DiffieHellman") == []
    assert "Masker" in c.types_held("alice") and "Masker" in c.types_held("bob")
    assert "Masker" not in c.types_held("carol")
    # the stand-in really refuses a client's datum
    with pytest.raises(fs.RevealRefused):
        fs.reveal(_put(c.pyu("alice"), np.ones(3)))


def test_dh_agreement_inside_the_parties(cpu_cluster):
    """No explicit seeds: the pair seeds come from a DH exchange of public
    keys; the sum still equals the oracle's (the masks cancel)."""
    from sfl_amd.compat import secretflow as hip

    c = cpu_cluster
    c.reveals.clear()
    agg = hip.SecureAggregator(c.pyu("carol"), [c.pyu(n) for n in NAMES], reveal=fs.reveal)
    rng = np.random.default_rng(11)
    xs = [(rng.standard_normal(1000) * 0.1).astype(np.float32) for _ in NAMES]
    for rnd in range(2):
        out = agg.average([_put(c.pyu(n), x) for n, x in zip(NAMES, xs)], axis=0, weights=[3, 5])
        exp = o.decode(o.server_sum([o.quantize(x, w) for x, w in zip(xs, [3, 5])]), divisor=8)
        assert np.array_equal(fs.reveal(out), exp)
        recv = [fs.reveal(m).u64 for m in agg.last_masked]
        # masked vectors are not the quantized ones (the masks are there) ...
        assert not np.array_equal(recv[0], o.quantize(xs[0], 3))
    assert [p for p, _ in c.reveals if p != "carol"] == ["alice", "bob"]
    assert _driver_holds("Masker", "DiffieHellman") == []


def test_argument_checks_before_any_party_work(cpu_cluster):
    from sfl_amd.compat import secretflow as hip

    c = cpu_cluster
    alice, bob, carol = (c.pyu(n) for n in NAMES + ["carol"])
    agg = hip.SecureAggregator(carol, [alice, bob], reveal=fs.reveal)
    with pytest.raises(TypeError):
        hip.SecureAggregator(object(), [alice])
    with pytest.raises(AssertionError, match="empty"):
        agg.sum([], axis=0)
    data = [_put(alice, np.ones(3)), _put(bob, np.ones(3))]
    with pytest.raises(AssertionError, match="not a participant"):
        agg.sum([_put(carol, np.zeros(3)), data[1]], axis=0)
    with pytest.raises(AssertionError, match="Device of weight does not match"):
        agg.average(data, axis=0, weights=[_put(bob, 1), _put(bob, 2)])
    with pytest.raises(AssertionError, match="Length of the weights"):
        agg.average(data, axis=0, weights=[1])
    with pytest.raises(AssertionError, match="every participant"):
        agg.sum([data[0]], axis=0)


# ------------------------------------------------------------------ install()
_SUBCLASS_SRC = '''
from secretflow.security import SecureAggregator


class FedGenLike(SecureAggregator):
    """The reference's subclass pattern (stateful_fedgen_aggregator.py:23-59)."""

    def __init__(self, device, participants, server_actor, fxp_bits=18):
        super().__init__(device, participants, fxp_bits)
        self.server_actor = server_actor

    def average(self, data, axis=None, weights=None):
        avg = super().average(data, axis, None)
        return self._device(lambda x: {"model_params": x})(avg)
'''


def _define_subclass():
    ns = {}
    exec(compile(_SUBCLASS_SRC, "<fedgen_like>", "exec"), ns)
    return ns["FedGenLike"]


def test_install_rebinds_both_import_paths(monkeypatch):
    from sfl_amd.compat import secretflow as hip

    mods = fs.installed_into(monkeypatch)
    rebound = hip.install()
    assert mods["secretflow.security"].SecureAggregator is hip.SecureAggregator
    assert mods["secretflow.security.aggregation"].SecureAggregator is hip.SecureAggregator
    assert len(rebound) == 2
    assert issubclass(_define_subclass(), hip.SecureAggregator)


def test_install_after_a_subclass_raises(monkeypatch):
    from sfl_amd.compat import secretflow as hip

    fs.installed_into(monkeypatch)
    early = _define_subclass()  # subclasses the placeholder
    with pytest.raises(RuntimeError, match="FedGenLike"):
        hip.install()
    assert not issubclass(early, hip.SecureAggregator)


def test_subclass_defined_after_install_aggregates(monkeypatch, cpu_cluster):
    from sfl_amd.compat import secretflow as hip

    fs.installed_into(monkeypatch)
    hip.install()
    c = cpu_cluster
    agg = _define_subclass()(c.pyu("carol"), [c.pyu(n) for n in NAMES], server_actor=None)
    x = [np.arange(6, dtype=np.float32).reshape(2, 3) * (k + 1) for k in range(2)]
    out = agg.average([_put(c.pyu(n), v) for n, v in zip(NAMES, x)], axis=0)
    got = fs.reveal(out)["model_params"]
    exp = o.decode(o.server_sum([o.quantize(v.reshape(-1)) for v in x]), divisor=2)
    assert np.array_equal(got.reshape(-1), exp)


@pytest.mark.skipif(not os.path.exists(REF_SUBCLASS), reason="reference checkout absent")
def test_reference_stateful_fedgen_aggregator_after_install(monkeypatch, cpu_cluster):
    """The reference's own StatefulFedGenAggregator source, loaded after
    install() into the stand-in secretflow package: its base is the drop-in
    and its weight-less average runs through the parties."""
    from sfl_amd.compat import secretflow as hip

    fs.installed_into(monkeypatch)
    hip.install()
    spec = importlib.util.spec_from_file_location("ref_stateful_fedgen_aggregator", REF_SUBCLASS)
    mod = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(mod)
    cls = mod.StatefulFedGenAggregator
    assert issubclass(cls, hip.SecureAggregator)
    c = cpu_cluster
    agg = cls(c.pyu("carol"), [c.pyu(n) for n in NAMES], server_actor=None)
    x = [[np.full((2, 2), 0.25 * (k + 1), np.float32), np.arange(3, dtype=np.float32)] for k in range(2)]
    out = agg.average([_put(c.pyu(n), v) for n, v in zip(NAMES, x)], axis=0)
    got = fs.reveal(out)
    assert isinstance(got, list) and len(got) == 2
    flat = [np.concatenate([a.reshape(-1) for a in v]) for v in x]
    exp = o.decode(o.server_sum([o.quantize(v) for v in flat]), divisor=2)
    assert np.array_equal(_flat(got), exp)


# ----------------------------------------------------------------------- GPU
@pytest.fixture(scope="module")
def gpu_cluster():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    c = _cluster(False)
    yield c
    c.close()


@pytest.mark.gpu
def test_gpu_contract_masks_in_each_party_process(gpu_cluster):
    """HIP sa_mask in alice's and bob's processes, sa_sum_u64 + sa_decode in
    carol's: the 7 AggregatorBase cases and every received masked vector
    bit-exact vs the oracle; only public keys revealed from the clients."""
    from sfl_amd.compat import secretflow as hip

    c = gpu_cluster
    seeds, pair = _seeds()
    c.reveals.clear()
    agg = hip.SecureAggregator(c.pyu("carol"), [c.pyu(n) for n in NAMES], reveal=fs.reveal, seeds=pair)
    _run_contract(c, agg, seeds, weights_on_device=True)
    assert [p for p, _ in c.reveals if p != "carol"] == ["alice", "bob"]
    assert _driver_holds("Masker", "DiffieHellman") == []


@pytest.mark.gpu
def test_gpu_subclass_after_install_and_rounds(monkeypatch, gpu_cluster):
    from sfl_amd.compat import secretflow as hip

    fs.installed_into(monkeypatch)
    hip.install()
    c = gpu_cluster
    agg = _define_subclass()(c.pyu("carol"), [c.pyu(n) for n in NAMES], server_actor=None)
    rng = np.random.default_rng(3)
    for _ in range(3):
        x = [(rng.standard_normal((64, 33)) * 0.05).astype(np.float32) for _ in NAMES]
        out = agg.average([_put(c.pyu(n), v) for n, v in zip(NAMES, x)], axis=0)
        got = fs.reveal(out)["model_params"]
        exp = o.decode(o.server_sum([o.quantize(v.reshape(-1)) for v in x]), divisor=2)
        assert np.array_equal(got.reshape(-1), exp)


# ------------------------------------------------------------ payload fuzz
def _random_payload(rng, n_layers, shapes, dtypes):
    out = []
    for sh, dt in zip(shapes, dtypes):
        if dt == np.int64:
            out.append(rng.integers(-2**20, 2**20, size=sh).astype(np.int64))
        else:
            out.append((rng.standard_normal(sh) * 10 ** rng.uniform(-3, 2)).astype(dt))
    return out


def _random_weight(rng, kind, shape):
    if kind == "none":
        return None
    if kind == "int":
        return int(rng.integers(1, 500))
    if kind == "float":
        return float(rng.uniform(0.1, 50))
    if kind == "np_float64":
        return np.float64(rng.uniform(0.1, 50))
    if kind == "np_int64":
        return np.int64(rng.integers(1, 500))
    if kind == "array":  # per-element weights (CHANGELOG.md:994), broadcast to every layer
        return rng.uniform(0.5, 5, size=shape).astype(np.float64)
    raise ValueError(kind)


def _expected_masked(layers, w, name, seeds, offset, fxp_bits=18):
    """The oracle per layer (each layer its own numpy arithmetic type), the
    layers' quantized values concatenated and masked from ``offset`` (the
    reference's per-layer rng.integers calls draw consecutive positions)."""
    q = np.concatenate([o.quantize(a, None if w is None else (np.broadcast_to(w, a.shape) if np.ndim(w) else w),
                                   fxp_bits).reshape(-1) for a in layers])
    return o.mask_client(q, name, seeds[name], offset)


def test_payload_fuzz_vs_oracle(cpu_cluster):
    """party.mask_payload / sum_decode over random payloads through the
    spawned-party drop-in: list / tuple / single arrays, float32 / float64 /
    int64 layers mixed in one payload, every weight kind (python int / float,
    numpy scalars under numpy 1.23.5 value-based casting, per-element arrays,
    device-object weights) -- every received masked vector and the result
    bit-exact vs the oracle, stream positions carried across 12 rounds."""
    _payload_fuzz(cpu_cluster, 2026, 12)


@pytest.mark.gpu
def test_gpu_payload_fuzz_vs_oracle(gpu_cluster):
    """The same fuzz with the HIP steps in the party processes (sa_mask with
    every compute type and weight form, sa_sum_u64 / sa_sum_f64 / sa_decode)."""
    _payload_fuzz(gpu_cluster, 77, 18)


def _payload_fuzz(c, seed, rounds):
    from sfl_amd.compat import secretflow as hip

    seeds, pair = _seeds()
    agg = hip.SecureAggregator(c.pyu("carol"), [c.pyu(n) for n in NAMES], reveal=fs.reveal, seeds=pair)
    rng = np.random.default_rng(seed)
    offset = 0
    kinds = ["none", "int", "float", "np_float64", "np_int64", "array"]
    for rnd in range(rounds):
        n_layers = int(rng.integers(1, 4))
        width = int(rng.integers(1, 7))
        shapes = [tuple(int(v) for v in rng.integers(1, 9, size=int(rng.integers(0, 3)))) + (width,)
                  for _ in range(n_layers)]
        container = ["array", "list", "tuple"][rnd % 3] if n_layers == 1 else ["list", "tuple"][rnd % 2]
        dts = [rng.choice([np.float32, np.float64, np.int64]) for _ in shapes]
        kind = kinds[rnd % len(kinds)]
        average = kind != "none" or rnd % 2 == 0
        payloads, ws = [], []
        for nm in NAMES:
            layers = _random_payload(rng, n_layers, shapes, dts)
            payloads.append(layers)
            ws.append(_random_weight(rng, kind, (width,)))
        objs = []
        for nm, layers in zip(NAMES, payloads):
            v = layers[0] if container == "array" else (tuple(layers) if container == "tuple" else layers)
            objs.append(_put(c.pyu(nm), v))
        if kind == "none":
            out = agg.average(objs, axis=0) if average else agg.sum(objs, axis=0)
            wl = None
        else:
            wobj = [_put(c.pyu(nm), w) if rnd % 4 == 1 and not np.ndim(w) else w for nm, w in zip(NAMES, ws)]
            out = agg.average(objs, axis=0, weights=wobj)
            wl = ws
        got = fs.reveal(out)
        masked = [_expected_masked(layers, None if wl is None else wl[i], nm, seeds, offset)
                  for i, (nm, layers) in enumerate(zip(NAMES, payloads))]
        recv = [fs.reveal(m) for m in agg.last_masked]
        for r, m in zip(recv, masked):
            assert np.array_equal(r.u64, m), (rnd, kind, dts)
        s = o.server_sum(masked)
        if not average:
            div = None
        elif wl is None:
            div = len(NAMES)
        elif np.ndim(wl[0]):
            div = np.concatenate([np.sum(np.stack([np.broadcast_to(w, sh).astype(np.float64) for w in wl]), axis=0)
                                  .reshape(-1) for sh in shapes])
        else:
            div = sum(wl)
        exp = o.decode(s, 18, div)
        flat = got.reshape(-1) if container == "array" else np.concatenate([np.asarray(g).reshape(-1) for g in got])
        assert np.array_equal(flat, exp), (rnd, kind, dts)
        if container != "array":
            assert isinstance(got, list if container == "list" else tuple) and len(got) == n_layers
            assert [np.shape(g) for g in got] == shapes
        offset += sum(int(np.prod(sh)) for sh in shapes)


def test_server_that_is_also_a_participant():
    """The notebook's own constructor, SecureAggregator(device=alice,
    participants=[alice, bob]) (secure_aggregation.ipynb:257-258): alice
    masks as a participant AND sums as the server; bob's values stay private."""
    from sfl_amd.compat import secretflow as hip

    c = fs.Cluster(NAMES, private=["bob"], init=_oracle_backend_init)
    try:
        seeds, pair = _seeds()
        alice, bob = c.pyu("alice"), c.pyu("bob")
        agg = hip.SecureAggregator(alice, [alice, bob], reveal=fs.reveal, seeds=pair)
        case = CONTRACT["sum_single"]
        xa, xb = _case_inputs(case)
        out = agg.sum([_put(alice, xa), _put(bob, xb)], axis=0)
        assert out.device == alice
        exp, _, _ = o.secure_sum([_cat(xa), _cat(xb)], NAMES, seeds=seeds)
        assert np.array_equal(fs.reveal(out).reshape(-1), exp)
        assert [p for p, _ in c.reveals if p == "bob"] == ["bob"]  # bob: his public key only
    finally:
        c.close()


def _notebook_kat(alice, bob, reveal):
    from sfl_amd.compat import secretflow as hip

    k = json.load(open(os.path.join(HERE, "golden", "notebook_kat.json")))
    agg = hip.SecureAggregator(device=alice, participants=[alice, bob], reveal=reveal)  # DH seeds
    a, b = _put(alice, np.array(k["arr0"])), _put(bob, np.array(k["arr1"]))
    s = reveal(agg.sum([a, b], axis=0))
    avg = reveal(agg.average([a, b], axis=0))
    assert s.dtype == np.float64
    assert np.abs(s - np.array(k["secure_sum"])).max() < 1e-8
    assert np.abs(avg - np.array(k["secure_average"])).max() < 1e-8


def test_notebook_kat_through_the_drop_in():
    """docs/developer/algorithm/secure_aggregation.ipynb cells 16-18 through
    the drop-in, parties as spawned processes (alice the server too)."""
    c = fs.Cluster(NAMES, private=["bob"], init=_oracle_backend_init)
    try:
        _notebook_kat(c.pyu("alice"), c.pyu("bob"), fs.reveal)
    finally:
        c.close()


@pytest.mark.gpu
def test_gpu_notebook_kat_through_the_drop_in_in_process():
    """The same with sfl_amd's in-process devices (the drop-in accepts any
    secretflow-shaped PYU) and the HIP steps."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.device import PYU, reveal

    _notebook_kat(PYU("alice", 0), PYU("bob", 0), reveal)


def _rejection_rounds(c):
    """The (alice, bob) pair stream draws a raw 0 at element 1000 of round 0
    (numpy's Generator.integers rejects it and takes the next draw): every
    masked vector the server receives and every result, over two rounds,
    equal numpy's own generators (OracleMaskers) -- the party resolves the
    rejection before its vector leaves, and its stream position moves one
    raw draw further."""
    from sfl_amd.compat import secretflow as hip
    from test_gpu_rejection import forced_zero_state

    state = {("alice", "bob"): forced_zero_state(1000)}
    agg = hip.SecureAggregator(c.pyu("carol"), [c.pyu(n) for n in NAMES], reveal=fs.reveal, seeds=state)
    ora = o.OracleMaskers(NAMES, state)
    rng = np.random.default_rng(12)
    n = 3001
    for rnd in range(2):
        xs = [(rng.standard_normal(n) * 1e-2).astype(np.float32) for _ in NAMES]
        out = agg.sum([_put(c.pyu(nm), x) for nm, x in zip(NAMES, xs)], axis=0)
        masked, ssum = ora.round(xs)
        assert np.array_equal(fs.reveal(out), o.decode(ssum)), rnd
        for r, m in zip([fs.reveal(m) for m in agg.last_masked], masked):
            assert np.array_equal(r.u64, m), rnd
        if rnd == 0:  # the round really held a rejection: numpy's stream differs from the plain raw + offset one
            plain = o.quantize(xs[0]) + (np.array(o.pcg64_raw_py(*state[("alice", "bob")], n), dtype=np.uint64)
                                         + np.uint64(o.MASK_OFFSET))
            assert not np.array_equal(masked[0], plain)
        # positions: round 1 starts one raw draw further for the pair
        assert [fs.reveal(m).positions for m in agg.last_masked] == [{"bob": rnd * (n + 1)}, {"alice": rnd * (n + 1)}]


def test_rejection_resolved_inside_the_party(cpu_cluster):
    _rejection_rounds(cpu_cluster)


@pytest.mark.gpu
def test_gpu_rejection_resolved_inside_the_party(gpu_cluster):
    _rejection_rounds(gpu_cluster)


def test_party_functions_leave_their_masker_argument_alone(monkeypatch):
    """mask_payload / agree return a NEW masker: with in-process devices a
    round that fails part-way must not have advanced the streams the
    aggregator still holds (an object store passes copies anyway)."""
    import party_oracle_backend
    from sfl_amd.security.aggregation import party as P

    monkeypatch.setattr(P, "_mask_vector", party_oracle_backend._mask_vector)
    m = P.new_masker("alice")
    m2 = P.agree(m, {"alice": m.public_key, "bob": P.new_masker("bob").public_key})
    assert m.peers == [] and m2.peers == ["bob"]
    wire, m3 = P.mask_payload(m2, np.ones(10, np.float32), None, None)
    assert m2.position("bob") == 0 and m3.position("bob") == 10 and wire.positions == {"bob": 0}


def test_lazy_runtime_failed_round_rolls_back():
    """under a lazy runtime (Ray, real secretflow) a party's
    failure inside ``average`` shows only when the result is resolved; the
    stored maskers are then failed futures and every later round fails.
    ``rollback()`` restores the maskers the failed round started from in
    every party, and the next round is bit-exact against the oracle at the
    positions after the last good round."""
    from sfl_amd.compat import secretflow as hip

    c = fs.Cluster(NAMES + ["carol"], private=NAMES, init=_oracle_backend_init, lazy=True)
    try:
        seeds, pair = _seeds()
        n = 37
        rng = np.random.default_rng(7)
        good = [[rng.standard_normal(n).astype(np.float32) for _ in NAMES] for _ in range(3)]

        def run(agg, xs):
            objs = [_put(c.pyu(nm), x) for nm, x in zip(NAMES, xs)]
            return agg.average(objs)

        def expect(xs, offset):
            return o.secure_average(xs, NAMES, seeds=seeds, offset=offset)[0]

        for use_rollback in (True, False):
            agg = hip.SecureAggregator(c.pyu("carol"), [c.pyu(nm) for nm in NAMES], reveal=fs.reveal, seeds=pair)
            assert np.array_equal(fs.reveal(run(agg, good[0])), expect(good[0], 0))
            # alice's payload has a type the masker refuses: under the lazy
            # runtime the call returns, the error surfaces at reveal
            bad = [np.ones(n, dtype=np.complex64), good[1][1]]
            res = run(agg, bad)
            with pytest.raises(fs.RemoteError, match="UpstreamError"):
                fs.reveal(res)
            if use_rollback:
                agg.rollback()
                agg.rollback()  # twice: a no-op
                assert np.array_equal(fs.reveal(run(agg, good[2])), expect(good[2], n))
            else:  # the failed futures poison every later round
                with pytest.raises(fs.RemoteError):
                    fs.reveal(run(agg, good[2]))
    finally:
        c.close()
