"""Parity of the HIP path (through the C-ABI) with the CPU oracle.

Bar: bit-exact for every integer output (masked vectors, masked sums, XOR
digests); decoded float64 equal to the oracle's float64 (same IEEE ops) and
within C * 2^-fxp of the float sum (the quantization tolerance).
"""
import ctypes

import numpy as np
import pytest

torch = pytest.importorskip("torch")

from oracle import secagg as o  # noqa: E402

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from sfl_amd import _lib as L

    L.lib()


def _K():
    from sfl_amd import kernels as K

    return K


def _L():
    from sfl_amd import _lib as L

    return L


def _streams(seeds, signs, offset):
    L = _L()
    return [(L.pcg64_advance(L.pcg64_from_seed(s), offset), sg, i) for i, (s, sg) in enumerate(zip(seeds, signs))]


def _oracle_masked(q, seeds, signs, offset):
    out = np.array(q, dtype=np.uint64).copy()
    for s, sg in zip(seeds, signs):
        m = o.mask_stream(s, out.size, offset)
        out = out + m if sg > 0 else out - m
    return out


def _u64(t):
    return _K().as_u64(t)


# ---------------------------------------------------------------------------
# single-client masking (sa_mask): the _Masker.mask replacement
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("n", [1, 3, 4, 5, 37, 1023, 1024, 1025, 4100, 70001])
@pytest.mark.parametrize("nstreams", [0, 1, 3, 7, 16, 17, 31])
def test_mask_f32_bit_exact(n, nstreams):
    K = _K()
    rng = np.random.default_rng(n * 100 + nstreams)
    x = (rng.standard_normal(n) * 5).astype(np.float32)
    seeds = [o.pair_seed(0, j + 1) for j in range(nstreams)]
    signs = [1 if j % 3 else -1 for j in range(nstreams)]
    offset = int(rng.integers(0, 1 << 40))
    exp = _oracle_masked(o.quantize(x), seeds, signs, offset)
    xt = torch.from_numpy(x).to(DEV)
    out = torch.empty(n, dtype=torch.int64, device=DEV)
    dig = torch.zeros(1, dtype=torch.int64, device=DEV)
    flags = torch.zeros(1, dtype=torch.int32, device=DEV)
    K.mask(xt, out, _streams(seeds, signs, offset), digest=dig, flags=flags)
    torch.cuda.synchronize()
    assert np.array_equal(_u64(out), exp)
    assert int(_u64(dig)[0]) == o.digest(exp)
    assert int(flags.item()) == 0


@pytest.mark.parametrize("case", ["f64", "i64", "f32_wvec_f64", "f32_scalar_w", "f64_scalar_w", "i64_int_w",
                                  "i64_float_w"])
def test_mask_other_types(case):
    K = _K()
    n = 2053
    rng = np.random.default_rng(11)
    seeds = [o.pair_seed(1, j) for j in (0, 2, 3)]
    signs = [-1, 1, 1]
    w, wvec, ct = None, None, None
    if case.startswith("f64"):
        x = rng.standard_normal(n) * 100
    elif case.startswith("i64"):
        x = rng.integers(-(1 << 20), 1 << 20, n)
    else:
        x = (rng.standard_normal(n) * 3).astype(np.float32)
    if case == "f32_wvec_f64":
        w = rng.integers(1, 50, n)  # int64 array -> float64 arithmetic
    elif case in ("f32_scalar_w", "f64_scalar_w"):
        w = 0.3
    elif case == "i64_int_w":
        w = 7
    elif case == "i64_float_w":
        w = 0.25
    q = o.quantize(x, w)
    ctype = {np.float32: torch.float32, np.float64: torch.float64, np.int64: torch.int64}
    cdt = (np.zeros(1, x.dtype) * (w if np.ndim(w) == 0 or w is None else np.zeros(1, np.asarray(w).dtype))).dtype \
        if w is not None else x.dtype
    ct = ctype[cdt.type]
    if w is not None and np.ndim(w):
        wvec = torch.from_numpy(np.asarray(w).astype(cdt)).to(DEV)
    exp = _oracle_masked(q, seeds, signs, 17)
    out = torch.empty(n, dtype=torch.int64, device=DEV)
    K.mask(torch.from_numpy(x).to(DEV), out, _streams(seeds, signs, 17),
           weight=1.0 if w is None or np.ndim(w) else w, weight_vec=wvec, compute_dtype=ct)
    torch.cuda.synchronize()
    assert np.array_equal(_u64(out), exp)


def test_quantize_edge_cases_bit_exact(golden_dir):
    K = _K()
    g = np.load(f"{golden_dir}/secagg_small.npz")
    for key in ("f32", "f64"):
        x = g[f"q_in_{key}"]
        out = torch.empty(x.size, dtype=torch.int64, device=DEV)
        K.mask(torch.from_numpy(x).to(DEV), out, [])
        torch.cuda.synchronize()
        assert np.array_equal(_u64(out), g[f"q_out_{key}"]), key


def test_golden_round_from_fixture(golden_dir):
    """3 parties, n=37, second round (offset 5): masked vectors, sum, decode."""
    K, L = _K(), _L()
    g = np.load(f"{golden_dir}/secagg_small.npz")
    names = ["alice", "bob", "carol"]
    seeds = o.seeds_for(names)
    off = int(g["round_offset"])
    n = g["round_x"].shape[1]
    masked = []
    for i, name in enumerate(names):
        peers = [p for p in names if p != name]
        st = [(L.pcg64_advance(L.pcg64_from_seed(seeds[name][p]), off), 1 if p > name else -1, j)
              for j, p in enumerate(peers)]
        out = torch.empty(n, dtype=torch.int64, device=DEV)
        K.mask(torch.from_numpy(g["round_x"][i]).to(DEV), out, st)
        masked.append(out)
    s = K.sum_u64(masked, torch.empty(n, dtype=torch.int64, device=DEV))
    dec = K.decode(s, torch.empty(n, dtype=torch.float64, device=DEV))
    torch.cuda.synchronize()
    assert np.array_equal(np.stack([_u64(m) for m in masked]), g["round_masked"])
    assert np.array_equal(_u64(s), g["round_sum"])
    assert np.array_equal(dec.cpu().numpy(), g["round_decoded"])


# ---------------------------------------------------------------------------
# fused co-located clients (sa_fused_clients)
# ---------------------------------------------------------------------------
def _fused_setup(C, n, offset, seed=0):
    L = _L()
    rng = np.random.default_rng(seed + C * 1000 + n)
    names = [f"party{c:02d}" for c in range(C)][::-1] if C % 2 else [f"party{c:02d}" for c in range(C)]
    xs = [(rng.standard_normal(n) * 0.01).astype(np.float32) for _ in range(C)]
    seeds = o.seeds_for(names)
    pair_gens, pair_signs = [], []
    for u in range(C):
        for v in range(u + 1, C):
            pair_gens.append(L.pcg64_advance(L.pcg64_from_seed(seeds[names[u]][names[v]]), offset))
            pair_signs.append(1 if names[v] > names[u] else -1)
    return names, xs, seeds, pair_gens, pair_signs


@pytest.mark.parametrize("C", [2, 3, 4, 5, 6, 7, 8])
@pytest.mark.parametrize("n", [5, 1024, 4099, 100003])
def test_fused_clients_bit_exact(C, n):
    K = _K()
    offset = 3 * n
    names, xs, seeds, pg, ps = _fused_setup(C, n, offset)
    masked = o.secure_masked(xs, names, seeds=seeds, offset=offset)
    s_exp = o.server_sum(masked)
    xt = [torch.from_numpy(x).to(DEV) for x in xs]
    s = torch.empty(n, dtype=torch.int64, device=DEV)
    dig = torch.zeros(C, dtype=torch.int64, device=DEV)
    mo = [torch.empty(n, dtype=torch.int64, device=DEV) for _ in range(C)]
    flags = torch.zeros(1, dtype=torch.int32, device=DEV)
    K.fused_clients(xt, [1.0] * C, pg, ps, [], 0, s, digests=dig, flags=flags, masked_outs=mo)
    torch.cuda.synchronize()
    assert np.array_equal(_u64(s), s_exp)
    for c in range(C):
        assert np.array_equal(_u64(mo[c]), masked[c]), c
    assert [int(v) for v in _u64(dig)] == [o.digest(m) for m in masked]
    assert int(flags.item()) == 0
    dec = K.decode(s, torch.empty(n, dtype=torch.float64, device=DEV))
    ref = o.decode(s_exp)
    assert np.array_equal(dec.cpu().numpy(), ref)
    assert np.abs(ref - np.sum(np.stack(xs).astype(np.float64), axis=0)).max() < C * 2.0**-18
    # the sum-only finish (no digests, no wire images: the bench's launch),
    # stored and accumulated
    s2 = torch.empty(n, dtype=torch.int64, device=DEV)
    K.fused_clients(xt, [1.0] * C, pg, ps, [], 0, s2, flags=flags)
    K.fused_clients(xt, [1.0] * C, pg, ps, [], 0, s2, accumulate=True)
    torch.cuda.synchronize()
    assert np.array_equal(_u64(s2), s_exp + s_exp)


@pytest.mark.parametrize("fxp", [0, 1, 7, 24, 31, 32, 40, 52, 62])
def test_fxp_bits_range(fxp):
    """Every fixed-point width the C-ABI accepts (0..62), not just the
    reference default 18: fused launch (pair sharing, digests, wire images,
    sum-only finish), per-client masking of f32 / f64 / int64 payloads with
    scalar weights, and the decode -- bit-exact vs the oracle.  Wide fxp
    sends every tile down the exact int64 path (|x*w*2^fxp| >= 2^31) and, at
    52+, past 2^63 (INT64_MIN, numpy's x86 astype); fxp 0 truncates most
    gradients to 0."""
    K = _K()
    C, n, off = 5, 4099, 7
    names, xs, seeds, pg, ps = _fused_setup(C, n, off, seed=fxp)
    xs = [x * np.float32(1 + 30 * c) for c, x in enumerate(xs)]  # magnitudes 1e-2 .. 1.2
    ws = [1.0, 0.5, 3.0, 0.1, 2.0]
    masked = o.secure_masked(xs, names, weights=ws, fxp_bits=fxp, seeds=seeds, offset=off)
    s_exp = o.server_sum(masked)
    s = torch.empty(n, dtype=torch.int64, device=DEV)
    dig = torch.zeros(C, dtype=torch.int64, device=DEV)
    mo = [torch.empty(n, dtype=torch.int64, device=DEV) for _ in range(C)]
    xt = [torch.from_numpy(x).to(DEV) for x in xs]
    K.fused_clients(xt, ws, pg, ps, [], 0, s, fxp_bits=fxp, digests=dig, masked_outs=mo)
    s2 = torch.empty(n, dtype=torch.int64, device=DEV)
    K.fused_clients(xt, ws, pg, ps, [], 0, s2, fxp_bits=fxp)
    dec = K.decode(s, torch.empty(n, dtype=torch.float64, device=DEV), fxp_bits=fxp, divisor=sum(ws))
    torch.cuda.synchronize()
    assert np.array_equal(_u64(s), s_exp)
    assert np.array_equal(_u64(s2), s_exp)
    for c in range(C):
        assert np.array_equal(_u64(mo[c]), masked[c]), c
    assert [int(v) for v in _u64(dig)] == [o.digest(m) for m in masked]
    assert np.array_equal(dec.cpu().numpy(), o.decode(s_exp, fxp, sum(ws)))
    # per-client masking of the other payload types at this width
    rng = np.random.default_rng(fxp)
    seeds1 = [o.pair_seed(2, j) for j in (0, 1, 3)]
    signs1 = [1, -1, 1]
    for x, w, ct in (((rng.standard_normal(n) * 50).astype(np.float64), 0.75, torch.float64),
                     (rng.integers(-(1 << 20), 1 << 20, n), 3, torch.int64),
                     ((rng.standard_normal(n) * 4).astype(np.float32), 0.3, torch.float32)):
        exp = _oracle_masked(o.quantize(x, w, fxp), seeds1, signs1, 99)
        out = torch.empty(n, dtype=torch.int64, device=DEV)
        K.mask(torch.from_numpy(x).to(DEV), out, _streams(seeds1, signs1, 99), weight=w, compute_dtype=ct,
               fxp_bits=fxp)
        torch.cuda.synchronize()
        assert np.array_equal(_u64(out), exp), ct


@pytest.mark.parametrize("C", [4, 8])
def test_fused_mixed_fast_and_exact_tiles(C):
    """A few scattered values that leave the int32 conversion (|x*w*2^fxp| >=
    2^31, +-inf, NaN) send their tiles down the exact int64 path while every
    other tile of the launch takes the one-v_cvt fast path: both bit-exact."""
    K = _K()
    n = 300_007
    names, xs, seeds, pg, ps = _fused_setup(C, n, 0, seed=C)
    rng = np.random.default_rng(100 + C)
    idx = rng.choice(n, 48, replace=False)
    bad = np.array([3e9, -3e9, np.inf, -np.inf, np.nan, 8192.0, -8192.0, 8191.999], np.float32)
    xs[1][idx] = bad[np.arange(idx.size) % bad.size]
    masked = o.secure_masked(xs, names, seeds=seeds)
    s = torch.empty(n, dtype=torch.int64, device=DEV)
    dig = torch.zeros(C, dtype=torch.int64, device=DEV)
    mo = [torch.empty(n, dtype=torch.int64, device=DEV) for _ in range(C)]
    K.fused_clients([torch.from_numpy(x).to(DEV) for x in xs], [1.0] * C, pg, ps, [], 0, s, digests=dig,
                    masked_outs=mo)
    torch.cuda.synchronize()
    assert np.array_equal(_u64(s), o.server_sum(masked))
    for c in range(C):
        assert np.array_equal(_u64(mo[c]), masked[c]), c
    assert [int(v) for v in _u64(dig)] == [o.digest(m) for m in masked]


def test_fused_accumulate_and_weights():
    K = _K()
    C, n = 4, 3001
    names, xs, seeds, pg, ps = _fused_setup(C, n, 0, seed=5)
    w = [128.0 * (c + 1) for c in range(C)]
    masked = o.secure_masked(xs, names, weights=[int(v) for v in w], seeds=seeds)
    exp = o.server_sum(masked)
    base = np.random.default_rng(1).integers(0, 2**63, n).astype(np.uint64)
    s = torch.from_numpy(base.view(np.int64).copy()).to(DEV)
    K.fused_clients([torch.from_numpy(x).to(DEV) for x in xs], w, pg, ps, [], 0, s, accumulate=True)
    torch.cuda.synchronize()
    assert np.array_equal(_u64(s), base + exp)


def test_fused_with_cross_streams_matches_per_client():
    """Shape of one GPU of a 2-GPU split: 2 local clients of 4, 2 cross
    streams each -- equals the sum of those clients' masked vectors."""
    K, L = _K(), _L()
    n = 9999
    names = ["a", "b", "c", "d"]
    seeds = o.seeds_for(names)
    rng = np.random.default_rng(3)
    xs = [(rng.standard_normal(n)).astype(np.float32) for _ in names]
    masked = o.secure_masked(xs, names, seeds=seeds, offset=11)
    local = [0, 1]
    pg = [L.pcg64_advance(L.pcg64_from_seed(seeds["a"]["b"]), 11)]
    ps = [1]
    cross = []
    for u in local:
        for p in ("c", "d"):
            cross.append((L.pcg64_advance(L.pcg64_from_seed(seeds[names[u]][p]), 11),
                          1 if p > names[u] else -1, 0))
    s = torch.empty(n, dtype=torch.int64, device=DEV)
    dig = torch.zeros(2, dtype=torch.int64, device=DEV)
    K.fused_clients([torch.from_numpy(xs[u]).to(DEV) for u in local], [1.0, 1.0], pg, ps, cross, 2, s,
                    digests=dig)
    torch.cuda.synchronize()
    assert np.array_equal(_u64(s), masked[0] + masked[1])
    assert [int(v) for v in _u64(dig)] == [o.digest(masked[0]), o.digest(masked[1])]


# ---------------------------------------------------------------------------
# server kernels
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("k", [1, 2, 8, 33, 70])
@pytest.mark.parametrize("n", [1, 2, 7, 4096, 12345])
def test_sum_u64(k, n):
    K = _K()
    rng = np.random.default_rng(k * n)
    ins = [rng.integers(0, 2**64 - 1, n, dtype=np.uint64) for _ in range(k)]
    ts = [torch.from_numpy(a.view(np.int64).copy()).to(DEV) for a in ins]
    out = K.sum_u64(ts, torch.empty(n, dtype=torch.int64, device=DEV))
    torch.cuda.synchronize()
    assert np.array_equal(_u64(out), o.server_sum(ins))


def test_decode_and_divisors():
    K = _K()
    n = 5003
    rng = np.random.default_rng(9)
    s = rng.integers(0, 2**64 - 1, n, dtype=np.uint64)
    s[:4] = [0, 2**63, 2**63 - 1, 2**64 - 1]
    st = torch.from_numpy(s.view(np.int64).copy()).to(DEV)
    for div in (1.0, 3.0, 640.0, 0.1):
        out = K.decode(st, torch.empty(n, dtype=torch.float64, device=DEV), divisor=div)
        torch.cuda.synchronize()
        assert np.array_equal(out.cpu().numpy(), o.decode(s, 18, div if div != 1.0 else None)), div
    dv = rng.integers(1, 100, n).astype(np.float64)
    out = K.decode(st, torch.empty(n, dtype=torch.float64, device=DEV), divisor_vec=torch.from_numpy(dv).to(DEV))
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), o.decode(s, 18, dv))


@pytest.mark.parametrize("n", [1, 2, 3, 7, 1024, 4099, 262_147, 3_000_001])
@pytest.mark.parametrize("shift", [0, 1])
def test_server_kernels_sizes_and_alignment(n, shift):
    """k_decode / k_sum_f64 / k_sum_u64 take 16-B accesses with 4 in flight
    per lane (an unrolled body, a remainder loop and an odd last element);
    sub-vectors at odd element offsets (8-B aligned only) take the one-element
    kernels.  Every size and alignment bit-exact vs the oracle / numpy."""
    K = _K()
    rng = np.random.default_rng(n + 7 * shift)
    s = rng.integers(0, 2**64 - 1, n, dtype=np.uint64)
    st = torch.from_numpy(s.view(np.int64).copy()).to(DEV)
    # shift: the buffers start one element into a fresh allocation
    sb = torch.empty(n + 1, dtype=torch.int64, device=DEV)
    sb[shift:shift + n] = st
    sv = sb[shift:shift + n]
    ob = torch.full((n + 1,), float("nan"), dtype=torch.float64, device=DEV)
    out = ob[shift:shift + n]
    K.decode(sv, out, divisor=3.0)
    dv = rng.integers(1, 100, n).astype(np.float64)
    dvb = torch.empty(n + 1, dtype=torch.float64, device=DEV)
    dvb[shift:shift + n] = torch.from_numpy(dv).to(DEV)
    out2 = torch.empty(n + 1, dtype=torch.float64, device=DEV)[shift:shift + n]
    K.decode(sv, out2, divisor_vec=dvb[shift:shift + n])
    ws = [rng.standard_normal(n) for _ in range(3)]
    wb = []
    for w in ws:
        b = torch.empty(n + 1, dtype=torch.float64, device=DEV)
        b[shift:shift + n] = torch.from_numpy(w).to(DEV)
        wb.append(b[shift:shift + n])
    fs = K.sum_f64(wb, torch.empty(n + 1, dtype=torch.float64, device=DEV)[shift:shift + n])
    torch.cuda.synchronize()
    assert np.array_equal(out.cpu().numpy(), o.decode(s, 18, 3.0))
    assert np.isnan(ob[(n if shift == 0 else 0)].item())  # nothing written past the vector
    assert np.array_equal(out2.cpu().numpy(), o.decode(s, 18, dv))
    assert np.array_equal(fs.cpu().numpy(), (ws[0] + ws[1]) + ws[2])
    if shift == 0:  # sa_sum_u64 needs 16-B aligned buffers
        ins = [torch.from_numpy(rng.integers(0, 2**64 - 1, n, dtype=np.uint64).view(np.int64)).to(DEV)
               for _ in range(5)]
        got = K.sum_u64(ins, torch.empty(n, dtype=torch.int64, device=DEV))
        torch.cuda.synchronize()
        assert np.array_equal(_u64(got), o.server_sum([_u64(t) for t in ins]))


def test_prg_zero_draw_is_flagged():
    """Force a raw PCG64 draw of 0 (hi == lo after the step) at element 5:
    numpy's Lemire bounded draw would reject it, so the kernel must flag."""
    K, L = _K(), _L()
    A = o.PCG64_MULT
    M = (1 << 128) - 1
    inc = (12345 << 1) | 1
    target = (0xDEADBEEF << 64) | 0xDEADBEEF  # hi == lo -> xsl-rr output 0
    ainv = pow(A, -1, 1 << 128)
    s = ((target - inc) * ainv) & M  # state before the draw that yields 0
    # walk back 5 steps so the zero lands on element 5
    for _ in range(5):
        s = ((s - inc) * ainv) & M
    g = L.PCG64.of(s, inc)
    assert o.pcg64_raw_py(s, inc, 6)[5] == 0
    out = torch.empty(64, dtype=torch.int64, device=DEV)
    flags = torch.zeros(1, dtype=torch.int32, device=DEV)
    K.mask(torch.zeros(64, device=DEV), out, [(g, 1, 0)], flags=flags)
    torch.cuda.synchronize()
    assert int(flags.item()) & L.SA_FLAG_PRG_REJECT


# ---------------------------------------------------------------------------
# full-size properties (BASELINE configs): too big for the oracle, so check
# mask cancellation, fused == per-client (wire) path, and oracle spot checks
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("C,n", [(4, 10_000_000), (8, 20_000_000), (8, 100_000_000)])
def test_full_size_properties(C, n):
    K, L = _K(), _L()
    names = [f"client{c}" for c in range(C)]
    seeds = o.seeds_for(names)
    xs = [torch.randn(n, device=DEV, dtype=torch.float32) * 1e-2 for _ in range(C)]
    pg, ps = [], []
    for u in range(C):
        for v in range(u + 1, C):
            pg.append(L.pcg64_from_seed(seeds[names[u]][names[v]]))
            ps.append(1 if names[v] > names[u] else -1)
    s = torch.empty(n, dtype=torch.int64, device=DEV)
    dig = torch.zeros(C, dtype=torch.int64, device=DEV)
    flags = torch.zeros(1, dtype=torch.int32, device=DEV)
    K.fused_clients(xs, [1.0] * C, pg, ps, [], 0, s, digests=dig, flags=flags)
    # (1) masks cancel: sum of unmasked quantized vectors
    q_sum = torch.zeros(n, dtype=torch.int64, device=DEV)
    qbuf = torch.empty(n, dtype=torch.int64, device=DEV)
    for x in xs:
        K.mask(x, qbuf, [], sum_accum=q_sum)
    # (2) the wire path: each client's masked vector, then the server sum
    wire = []
    wdig = torch.zeros(C, dtype=torch.int64, device=DEV)
    for c in range(C):
        st = [(L.pcg64_from_seed(seeds[names[c]][p]), 1 if p > names[c] else -1, j)
              for j, p in enumerate(q for q in names if q != names[c])]
        out = torch.empty(n, dtype=torch.int64, device=DEV)
        K.mask(xs[c], out, st, digest=wdig[c:c + 1])
        wire.append(out)
    s2 = K.sum_u64(wire, torch.empty(n, dtype=torch.int64, device=DEV))
    # the bench's launch: no digests, no wire images (the sum-only finish)
    s3 = torch.empty(n, dtype=torch.int64, device=DEV)
    K.fused_clients(xs, [1.0] * C, pg, ps, [], 0, s3)
    torch.cuda.synchronize()
    assert torch.equal(s, q_sum)
    assert torch.equal(s, s2)
    assert torch.equal(s, s3)
    assert torch.equal(dig, wdig)
    assert int(flags.item()) == 0
    # (3a) the bench's own launch (sum-only <C,0,4>) pinned to the oracle
    # directly: >= 8 windows of 4096 element positions (both ends, the
    # middle, random offsets), every pair stream jumped to the window start
    from oracle_windows import check_partial_sum_windows

    assert check_partial_sum_windows(s3, xs, list(range(C)), names, seeds, 0, k_random=6, seed=C) >= 8 * 4096
    # (3) oracle spot checks of individual masked elements at far offsets
    rng = np.random.default_rng(0)
    idx = np.concatenate([[0, 1, n - 1], rng.integers(0, n, 20)])
    xh = [x[idx].cpu().numpy() for x in xs]
    for c in range(C):
        got = _u64(wire[c][idx])
        for t, i in enumerate(idx):
            v = int(o.quantize(xh[c][t:t + 1])[0])
            for p in names:
                if p != names[c]:
                    m = int(o.mask_stream(seeds[names[c]][p], 1, int(i))[0])
                    v = (v + m) & o.U64 if p > names[c] else (v - m) & o.U64
            assert int(got[t]) == v
    # (4) decoded sum within C * 2^-18 of the float sum
    dec = K.decode(s, torch.empty(n, dtype=torch.float64, device=DEV))
    fsum = torch.stack(xs).double().sum(0)
    assert float((dec - fsum).abs().max()) < C * 2.0**-18


def test_fused_fallback_for_uninstantiated_shape():
    """32 clients, 4 on this GPU (config 5 per-rank shape): 6 internal pairs +
    28 cross streams each exceed one fused launch; the wrapper falls back to
    per-client masking with accumulation -- bit-identical to the oracle."""
    K = _K()
    from sfl_amd.parallel_sum import plan_generators, plan_rank

    C, W, n = 32, 8, 5003
    names = [f"c{i:02d}" for i in range(C)]
    seeds = o.seeds_for(names)
    plan = plan_rank(names, W, 3)
    seed_of = lambda u, v: seeds[names[u]][names[v]]  # noqa: E731
    pg, ps, cross = plan_generators(plan, seed_of, offset=7)
    rng = np.random.default_rng(2)
    xs = [(rng.standard_normal(n) * 1e-2).astype(np.float32) for _ in range(C)]
    masked = o.secure_masked(xs, names, seeds=seeds, offset=7)
    s = torch.empty(n, dtype=torch.int64, device=DEV)
    dig = torch.zeros(len(plan.clients), dtype=torch.int64, device=DEV)
    K.fused_clients([torch.from_numpy(xs[c]).to(DEV) for c in plan.clients], [1.0] * len(plan.clients), pg, ps,
                    cross, plan.n_cross, s, digests=dig)
    torch.cuda.synchronize()
    exp = np.zeros(n, dtype=np.uint64)
    for c in plan.clients:
        exp += masked[c]
    assert np.array_equal(_u64(s), exp)
    assert [int(v) for v in _u64(dig)] == [o.digest(masked[c]) for c in plan.clients]


def test_fused_more_than_8_clients_falls_back():
    """12 clients on one GPU (config 5 run on one GPU is 32): more co-located
    clients than one launch holds -> SA_ERR_UNSUPPORTED -> per-client masking
    with accumulation, bit-identical to the oracle."""
    K = _K()
    C, n = 12, 4099
    names, xs, seeds, pg, ps = _fused_setup(C, n, 9)
    masked = o.secure_masked(xs, names, seeds=seeds, offset=9)
    s = torch.empty(n, dtype=torch.int64, device=DEV)
    dig = torch.zeros(C, dtype=torch.int64, device=DEV)
    K.fused_clients([torch.from_numpy(x).to(DEV) for x in xs], [1.0] * C, pg, ps, [], 0, s, digests=dig)
    torch.cuda.synchronize()
    assert np.array_equal(_u64(s), o.server_sum(masked))
    assert [int(v) for v in _u64(dig)] == [o.digest(m) for m in masked]


@pytest.mark.parametrize("C", [9, 12, 13, 16, 21, 32])
@pytest.mark.parametrize("n", [5, 4099, 70001])
def test_fused_many_pair_shared_bit_exact(C, n):
    """More co-located clients than one launch holds and only the sum wanted
    (no digests / wire images): fused_clients routes to the pair-shared
    schedule -- groups of up to 8 through sa_fused_clients, every pair of
    quads in different groups through sa_fused_bipartite, a short last quad
    padded -- so every pair stream is expanded once.  The sum equals the
    oracle's bit for bit (weighted clients, mixed pair signs), also
    accumulated onto a prior sum, and the PRG flag stays clear."""
    K = _K()
    offset = 5 * n + 3
    names, xs, seeds, pg, ps = _fused_setup(C, n, offset)
    w = [1 + c % 3 for c in range(C)]
    exp = o.server_sum(o.secure_masked(xs, names, weights=w, seeds=seeds, offset=offset))
    xt = [torch.from_numpy(x).to(DEV) for x in xs]
    s = torch.empty(n, dtype=torch.int64, device=DEV)
    flags = torch.zeros(1, dtype=torch.int32, device=DEV)
    K.fused_clients(xt, [float(v) for v in w], pg, ps, [], 0, s, flags=flags)
    base = np.random.default_rng(C).integers(0, 2**63, n, dtype=np.uint64)
    acc = torch.from_numpy(base.view(np.int64).copy()).to(DEV)
    K.fused_many(xt, [float(v) for v in w], pg, ps, acc, accumulate=True)
    torch.cuda.synchronize()
    assert np.array_equal(_u64(s), exp)
    assert np.array_equal(_u64(acc), base + exp)
    assert int(flags.item()) == 0


def test_fused_many_full_size_32_clients():
    """Config 5's 32 clients on one GPU at 64M elements each (the bench runs
    256M): the pair-shared schedule's sum equals the sum of the unmasked
    quantized vectors (every pair's masks cancel) and the per-client path's
    sum (both ends of every pair drawn separately, with digests), bit for
    bit; no PRG flag."""
    K, L = _K(), _L()
    C, n = 32, 64 * 2**20 + 77
    names = [f"client{c:02d}" for c in range(C)]
    seeds = o.seeds_for(names)
    xs = [torch.randn(n, device=DEV, dtype=torch.float32) * 1e-2 for _ in range(C)]
    pg, ps = [], []
    for u in range(C):
        for v in range(u + 1, C):
            pg.append(L.pcg64_advance(L.pcg64_from_seed(seeds[names[u]][names[v]]), 7 * n))
            ps.append(1 if names[v] > names[u] else -1)
    s = torch.empty(n, dtype=torch.int64, device=DEV)
    flags = torch.zeros(1, dtype=torch.int32, device=DEV)
    K.fused_clients(xs, [1.0] * C, pg, ps, [], 0, s, flags=flags)  # -> fused_many
    q_sum = torch.zeros(n, dtype=torch.int64, device=DEV)
    qbuf = torch.empty(n, dtype=torch.int64, device=DEV)
    for x in xs:
        K.mask(x, qbuf, [], sum_accum=q_sum)
    s2 = torch.empty(n, dtype=torch.int64, device=DEV)
    dig = torch.zeros(C, dtype=torch.int64, device=DEV)
    K.fused_clients(xs, [1.0] * C, pg, ps, [], 0, s2, digests=dig)  # per-client path
    torch.cuda.synchronize()
    assert torch.equal(s, q_sum)
    assert torch.equal(s, s2)
    assert int(flags.item()) == 0


def test_fused_many_padding_streams_cancel():
    """A bipartite launch whose slots are all padding (no input, dummy pair
    streams) leaves the sum unchanged: the padded pairs' masks cancel."""
    K, L = _K(), _L()
    n = 10_007
    base = np.random.default_rng(5).integers(0, 2**64 - 1, n, dtype=np.uint64)
    s = torch.from_numpy(base.view(np.int64).copy()).to(DEV)
    clients = (L.LocalClient * 8)()
    for c in range(8):
        clients[c].x, clients[c].weight, clients[c].masked_out = None, 1.0, None
    gens = (L.PCG64 * 16)(*[L.pcg64_from_seed(1000 + p) for p in range(16)])
    signs = (ctypes.c_int8 * 16)(*[1 if p % 3 else -1 for p in range(16)])
    L.check(L.lib().sa_fused_bipartite(clients, L.SA_F32, n, 18, gens, signs, ctypes.c_void_p(s.data_ptr()), 1, None,
                                       ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)), "bipartite")
    torch.cuda.synchronize()
    assert np.array_equal(_u64(s), base)


def test_chunked_launch_past_4gib():
    """Vectors longer than one launch's 32-bit buffer offsets (2^29 - 1024
    u64) are cut into chunks whose streams resume at the chunk offset: the
    masked elements either side of the boundary and at the tail match the
    oracle, and the fused sum equals the per-client masked sum."""
    K, L = _K(), _L()
    chunk = (1 << 29) - 1024
    n = (1 << 29) + 3001
    names = ["p0", "p1"]
    seeds = o.seeds_for(names)
    sd = seeds["p0"]["p1"]
    xs = [torch.randn(n, device=DEV, dtype=torch.float32) * 1e-2 for _ in names]
    outs = [torch.empty(n, dtype=torch.int64, device=DEV) for _ in names]
    wsum = torch.zeros(n, dtype=torch.int64, device=DEV)
    wdig = torch.zeros(2, dtype=torch.int64, device=DEV)
    for c, sign in ((0, 1), (1, -1)):
        K.mask(xs[c], outs[c], [(L.pcg64_from_seed(sd), sign, 0)], sum_accum=wsum, digest=wdig[c:c + 1])
    s = torch.empty(n, dtype=torch.int64, device=DEV)
    dig = torch.zeros(2, dtype=torch.int64, device=DEV)
    mo = [torch.empty(n, dtype=torch.int64, device=DEV) for _ in names]
    K.fused_clients(xs, [1.0, 1.0], [L.pcg64_from_seed(sd)], [1], [], 0, s, digests=dig, masked_outs=mo)
    torch.cuda.synchronize()
    assert torch.equal(s, wsum)
    assert torch.equal(dig, wdig)
    for c in range(2):
        assert torch.equal(mo[c], outs[c])
    for lo in (0, chunk - 40, n - 40):
        m = o.mask_stream(sd, 40, lo)
        q0 = o.quantize(xs[0][lo:lo + 40].cpu().numpy())
        assert np.array_equal(_u64(outs[0][lo:lo + 40]), q0.view(np.uint64) + m), lo
    del xs, outs, mo
    torch.cuda.empty_cache()


def test_launches_capture_into_a_graph():
    """include/sfl_sa.h promises launch functions that never allocate, copy
    or synchronise: the fused masking launch and the decode captured into a
    HIP graph (torch.cuda.CUDAGraph on ROCm) replay to the eager results."""
    K, L = _K(), _L()
    C, n = 4, 100_003
    names, xs, seeds, pg, ps = _fused_setup(C, n, 0)
    xd = [torch.from_numpy(x).to(DEV) for x in xs]
    s_e = torch.empty(n, dtype=torch.int64, device=DEV)
    d_e = torch.empty(n, dtype=torch.float64, device=DEV)
    K.fused_clients(xd, [1.0] * C, pg, ps, [], 0, s_e)
    K.decode(s_e, d_e, divisor=float(C))
    s_g = torch.zeros(n, dtype=torch.int64, device=DEV)
    d_g = torch.zeros(n, dtype=torch.float64, device=DEV)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        with torch.cuda.graph(g):
            K.fused_clients(xd, [1.0] * C, pg, ps, [], 0, s_g)
            K.decode(s_g, d_g, divisor=float(C))
    torch.cuda.current_stream().wait_stream(side)
    for _ in range(2):
        s_g.zero_()
        g.replay()
    torch.cuda.synchronize()
    assert torch.equal(s_g, s_e)
    assert torch.equal(d_g, d_e)
    masked = o.secure_masked(xs, names, seeds=seeds)
    assert np.array_equal(_u64(s_g), o.server_sum(masked))
