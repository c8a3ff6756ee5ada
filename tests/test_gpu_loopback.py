"""Loopback-socket party processes (BASELINE config 1 shape, SURVEY.md §8f
row 2): one spawned process per client masks on the GPU and ships raw u64
frames over 127.0.0.1; the server (this process) sums and decodes on the GPU.
Checked against the oracle: the received wire images equal the oracle's
masked vectors bit for bit, and the decoded results equal its float64."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")
from oracle import secagg as o  # noqa: E402

pytestmark = pytest.mark.gpu


def test_loopback_rounds_bit_exact_vs_oracle():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.loopback import run_loopback, synthetic_gradient

    names = ["alice", "bob", "carol"]
    n, rounds = 20_011, 2
    seeds = o.seeds_for(names)
    w = [3, 5, 8]
    res, timings, stats, masked = run_loopback(names, n, rounds, seeds=seeds, weights=w, average=True,
                                               keep_masked=True, verify_digest=True, timeout=300)
    for r in range(rounds):
        xs = [synthetic_gradient(c, n, r) for c in range(len(names))]
        exp, s, m = o.secure_average(xs, names, weights=w, seeds=seeds, offset=r * n)
        assert np.array_equal(res[r], exp), r
        for c in range(len(names)):
            assert np.array_equal(masked[r][c], m[c]), (r, c)
            assert stats[c][r]["result_xor"] == int(np.bitwise_xor.reduce(exp.view(np.uint64)))


def test_loopback_dh_seeds_sum():
    """Real DH agreement inside the party processes (seeds unknown to the
    test): the masked sum is PRG-independent, so the decoded sum still equals
    the oracle's."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.loopback import run_loopback, synthetic_gradient

    names = [f"p{i}" for i in range(4)]
    n = 4099
    res, _, _, masked = run_loopback(names, n, 1, keep_masked=True, timeout=300)
    xs = [synthetic_gradient(c, n, 0) for c in range(len(names))]
    q = [o.quantize(x) for x in xs]
    assert np.array_equal(res[0], o.decode(o.server_sum(q)))
    for c in range(len(names)):
        assert not np.array_equal(masked[0][c], q[c])  # masked on the wire


def test_loopback_chunked_streaming_multi_party_processes(monkeypatch):
    """Transfers larger than the staging chunk stream through the pinned
    rings on both sides; 4 parties hosted 2 per process (config 5 layout)."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    monkeypatch.setenv("SFL_LOOPBACK_CHUNK_ELEMS", "4096")
    from sfl_amd.loopback import run_loopback, synthetic_gradient

    names = [f"q{i}" for i in range(4)]
    n = 50_001
    seeds = o.seeds_for(names)
    res, _, _, masked = run_loopback(names, n, 2, seeds=seeds, keep_masked=True, verify_digest=True,
                                     parties_per_process=2, timeout=300)
    for r in range(2):
        xs = [synthetic_gradient(c, n, r) for c in range(len(names))]
        masked_o = o.secure_masked(xs, names, seeds=seeds, offset=r * n)
        assert np.array_equal(res[r], o.decode(o.server_sum(masked_o)))
        for c in range(len(names)):
            assert np.array_equal(masked[r][c], masked_o[c])


def test_loopback_client_reproduces_numpy_rejection():
    """A pair stream whose raw draw 777 is 0 (numpy rejects it): the client
    party moves its masked vector onto numpy's stream before sending, so the
    wire images (digest-verified) equal numpy's in both rounds."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from test_gpu_rejection import forced_zero_state

    from sfl_amd.loopback import run_loopback, synthetic_gradient

    names = ["alice", "bob", "carol"]
    n = 2048
    seeds = o.seeds_for(names)
    st = forced_zero_state(777)
    seeds["alice"]["carol"] = seeds["carol"]["alice"] = st
    res, _, _, masked = run_loopback(names, n, 2, seeds=seeds, keep_masked=True, verify_digest=True, timeout=300)
    pair = {(a, b): seeds[a][b] for a in names for b in names if a < b}
    ora = o.OracleMaskers(names, pair)
    for r in range(2):
        xs = [synthetic_gradient(c, n, r) for c in range(len(names))]
        m, ssum = ora.round(xs)
        assert np.array_equal(res[r], o.decode(ssum)), r
        for c in range(len(names)):
            assert np.array_equal(masked[r][c], m[c]), (r, c)


@pytest.mark.parametrize("send", ["copy", "sendfile"])
def test_loopback_chunks_without_result_copies(monkeypatch, send):
    """Both send modes over many chunks (masked vectors D2H into registered
    memfd pages chunk by chunk, each sent as it lands; the result D2H'd into
    the server's pages and broadcast from them), with no copy of the result
    kept by the server or the clients (keep_results=False: the clients
    receive it through a ring of two chunks and checksum it as it lands):
    every client received the oracle's float64 result, round after round,
    with the streams advancing."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.loopback import run_loopback, synthetic_gradient

    monkeypatch.setenv("SFL_LOOPBACK_SEND", send)  # the spawned clients inherit both
    monkeypatch.setenv("SFL_LOOPBACK_CHUNK_ELEMS", "8192")  # 9 chunks
    names = ["p0", "p1", "p2", "p3"]
    n, rounds = 70_001, 3
    seeds = o.seeds_for(names)
    res, _, stats, _ = run_loopback(names, n, rounds, seeds=seeds, keep_results=False, timeout=300)
    assert res == [None] * rounds
    for r in range(rounds):
        xs = [synthetic_gradient(c, n, r) for c in range(len(names))]
        exp = o.secure_sum(xs, names, seeds=seeds, offset=r * n)[0]
        want = int(np.bitwise_xor.reduce(exp.view(np.uint64)))
        assert [stats[c][r]["result_xor"] for c in range(len(names))] == [want] * len(names), r


def test_loopback_multi_gpu_placement_bit_exact():
    """run_loopback(gpus=[0, 0]): the placement path of the 8-GPU node
    (client process g on gpus[g % len(gpus)], the server on its own device
    context) on the one GPU of this box; wire images and results bit-exact
    vs the oracle, the placement recorded in the timings."""
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd.loopback import run_loopback, synthetic_gradient

    names = [f"g{i}" for i in range(4)]
    n, rounds = 30_011, 2
    seeds = o.seeds_for(names)
    res, timings, stats, masked = run_loopback(names, n, rounds, seeds=seeds, keep_masked=True, verify_digest=True,
                                               gpus=[0, 0], parties_per_process=1, timeout=300)
    assert timings[0]["placement"] == {"server_gpu": 0, "client_process_gpus": [0, 0, 0, 0],
                                       "parties_per_process": 1}
    for r in range(rounds):
        xs = [synthetic_gradient(c, n, r) for c in range(len(names))]
        exp, _, m = o.secure_sum(xs, names, seeds=seeds, offset=r * n)
        assert np.array_equal(res[r], exp), r
        for c in range(len(names)):
            assert np.array_equal(masked[r][c], m[c]), (r, c)
