"""The C-ABI used from plain C (tests/c_abi/abi_roundtrip.c: what a cgo /
JNI / N-API binding would do -- no Python or torch in the process): three
parties, sa_pcg64_from_seed -> sa_pcg64_advance -> sa_mask -> sa_sum_u64 ->
sa_decode on the GPU, then the same round through the blocking host-array
entries (sa_mask_host -> sa_sum_decode_host, sa_fused_clients_host_f32).
Its masked vectors and masked sum equal the numpy oracle bit for bit, its
decodes equal the oracle's float64, its digests the XOR of the oracle's
masked vectors."""
import os
import subprocess

import numpy as np
import pytest

from oracle import secagg as o

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BIN = os.path.join(ROOT, "sfl_amd", "lib", "abi_roundtrip")


def _inputs(n, parties=3):
    i = np.arange(n, dtype=np.uint64).astype(np.uint32)
    xs = []
    for c in range(parties):
        v = (i * np.uint32(2654435761) + np.uint32(97 * c)) % np.uint32(20001)
        xs.append((v.astype(np.int32) - 10000).astype(np.float32) / np.float32(1e6))
    return xs


@pytest.mark.parametrize("n", [1, 10007, 300001])
def test_plain_c_client_matches_oracle(tmp_path, n):
    torch = pytest.importorskip("torch")
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    if not os.path.exists(BIN):
        pytest.skip("abi_roundtrip not built (tests/c_abi/Makefile, run by __graft_entry__.build())")
    out = tmp_path / "out.bin"
    subprocess.run([BIN, str(out), str(n)], check=True, timeout=120, capture_output=True)
    raw = np.fromfile(out, dtype=np.uint64)
    assert int(raw[0]) == n
    masked = raw[1:1 + 3 * n].reshape(3, n)
    s = raw[1 + 3 * n:1 + 4 * n]
    dec = raw[1 + 4 * n:1 + 5 * n].view(np.float64)

    names = ["p0", "p1", "p2"]
    seeds = o.seeds_for(names)
    exp = o.secure_masked(_inputs(n), names, seeds=seeds, offset=5)
    for c in range(3):
        assert np.array_equal(masked[c], exp[c]), c
    s_exp = o.server_sum(exp)
    assert np.array_equal(s, s_exp)
    assert np.array_equal(dec, o.decode(s_exp))
    # the blocking host-array entries on the same round
    k = 1 + 5 * n
    masked_h = raw[k:k + 3 * n].reshape(3, n)
    dec_h = raw[k + 3 * n:k + 4 * n].view(np.float64)
    dig_h = raw[k + 4 * n:k + 4 * n + 3]
    dec_f = raw[k + 4 * n + 3:k + 5 * n + 3].view(np.float64)
    dig_f = raw[k + 5 * n + 3:k + 5 * n + 6]
    flags = raw[k + 5 * n + 6:k + 5 * n + 8]
    want_dig = [int(np.bitwise_xor.reduce(e)) for e in exp]
    for c in range(3):
        assert np.array_equal(masked_h[c], exp[c]), c
    assert np.array_equal(dec_h, o.decode(s_exp)) and np.array_equal(dec_f, o.decode(s_exp))
    assert [int(v) for v in dig_h] == want_dig and [int(v) for v in dig_f] == want_dig
    assert raw.size == k + 5 * n + 8 and not flags.any()
