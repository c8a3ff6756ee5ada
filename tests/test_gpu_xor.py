"""sa_xor_u64 (kernels.xor_digest): the XOR digest the server checks every
masked vector with -- every length around the kernel's 16-byte pairs and
4-way unroll, 8-byte-misaligned starts, accumulation into a non-zero
digest; and its streaming rate at a chunk's size (printed)."""
import numpy as np
import pytest

torch = pytest.importorskip("torch")

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")


@pytest.mark.parametrize("off", [0, 1])
@pytest.mark.parametrize("n", [1, 2, 3, 255, 256, 257, 1023, 524_289, 2_097_153, 12_500_001])
def test_xor_digest_bit_exact(n, off):
    from sfl_amd import kernels as K

    rng = np.random.default_rng(n + off)
    host = rng.integers(0, 2**63, n + off, dtype=np.int64) * 2 + 1
    dev = torch.from_numpy(host).to("cuda:0")
    seed = np.int64(0x1234_5678_9ABC_DEF)
    dig = torch.tensor([seed], dtype=torch.int64, device="cuda:0")
    K.xor_digest(dev[off:], dig)
    want = np.bitwise_xor.reduce(host[off:].view(np.uint64)) ^ np.uint64(seed)
    assert int(dig.cpu().numpy().view(np.uint64)[0]) == int(want)


def test_xor_digest_rate():
    from sfl_amd import kernels as K

    n = 12_500_000  # one 8-chunk sum_decode chunk of a 100M vector
    v = torch.randint(-2**62, 2**62, (n,), dtype=torch.int64, device="cuda:0")
    dig = torch.zeros(1, dtype=torch.int64, device="cuda:0")
    for _ in range(3):
        K.xor_digest(v, dig)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(20):
        K.xor_digest(v, dig)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / 20
    print(f"xor_digest: {n} words in {ms * 1e3:.1f} us, {8 * n / ms / 1e9:.2f} TB/s")
    assert ms > 0
