"""The CPU oracle pinned against the reference's own known answers and numpy.

oracle/secagg.py is test infrastructure; these tests check it before any GPU
result is compared to it:
  * the notebook KAT (docs/developer/algorithm/secure_aggregation.ipynb
    cells 7/17/18) — secure sum and average of two parties;
  * the AggregatorBase contract values
    (tests/security/aggregation/test_aggregator_base.py:21-160);
  * numpy's PCG64 / Generator.integers (the reference's PRG dependency);
  * the committed golden vectors (tests/golden/make_golden.py).
"""
import json
import os

import numpy as np
import pytest

from oracle import secagg as o


def test_notebook_kat(golden_dir):
    k = json.load(open(os.path.join(golden_dir, "notebook_kat.json")))
    a0, a1 = np.array(k["arr0"]), np.array(k["arr1"])
    dec, s, masked = o.secure_sum([a0, a1], k["parties"], k["fxp_bits"])
    # inputs printed to 8 digits -> residual ~5e-9 with trunc quantization
    assert np.abs(dec - np.array(k["secure_sum"])).max() < 1e-8
    avg, _, _ = o.secure_average([a0, a1], k["parties"], None, k["fxp_bits"])
    assert np.abs(avg - np.array(k["secure_average"])).max() < 1e-8
    # round-to-nearest would miss by ~7.6e-6: the KAT pins truncation
    rn = np.sum([np.round(a * 2**18) for a in (a0, a1)], axis=0) / 2**18
    assert np.abs(rn - np.array(k["secure_sum"])).max() > 1e-6
    assert dec.dtype == np.float64
    # masks really mask, and really cancel
    assert not np.array_equal(masked[0], o.quantize(a0))
    assert np.array_equal(s, o.quantize(a0) + o.quantize(a1))


def _contract(golden_dir):
    return json.load(open(os.path.join(golden_dir, "aggregator_contract.json")))


@pytest.mark.parametrize("case", ["sum_single", "sum_list", "avg_single", "avg_list",
                                  "avg_weights", "avg_list_weights", "avg_same_shape_weights"])
def test_aggregator_contract_values(golden_dir, case):
    c = _contract(golden_dir)[case]
    names = ["alice", "bob"]
    a, b = np.array(c["a"]), np.array(c["b"])
    layers = [(a[i], b[i]) for i in range(len(a))] if case.endswith("list") or "list_" in case else [(a, b)]
    w = c.get("weights")
    for li, (xa, xb) in enumerate(layers):
        if case.startswith("sum"):
            got, _, _ = o.secure_sum([xa, xb], names)
        else:
            ww = None if w is None else [np.array(w[0]), np.array(w[1])] if np.ndim(w[0]) else w
            got, _, _ = o.secure_average([xa, xb], names, ww)
        if "expect" in c:
            exp = np.array(c["expect"])
            exp = exp[li] if len(layers) > 1 else exp
        else:
            exp = np.average([xa, xb], axis=0, weights=np.array(w))
        np.testing.assert_almost_equal(got, exp, decimal=c["decimal"])


def test_pcg64_restatement_matches_numpy():
    for seed in [0, 7, o.pair_seed(1, 2), 2**100 + 5]:
        st, inc = o.pcg64_state(seed)
        bg = np.random.PCG64(seed)
        assert o.pcg64_raw_py(st, inc, 8) == [int(v) for v in bg.random_raw(8)]
        s2 = o.pcg64_jump_py(st, inc, 999_983)
        bg = np.random.PCG64(seed)
        bg.advance(999_983)
        assert s2 == bg.state["state"]["state"]
        # Generator.integers(int64.min, int64.max) == raw + (2^63 - 1)
        m = o.mask_stream(seed, 8, 999_983)
        raw = o.pcg64_raw_py(s2, inc, 8)
        assert [int(v) for v in m] == [(r + o.MASK_OFFSET) & o.U64 for r in raw]


def test_quantize_matches_numpy_astype_on_x86():
    x = np.array([0.3, -0.3, 1e30, -1e30, np.inf, np.nan, 2.0**-19, -(2.0**-17)], dtype=np.float32)
    with np.errstate(all="ignore"):
        ref = (x * (1 << 18)).astype(np.int64).astype(np.uint64)
    assert np.array_equal(ref, o.quantize(x))
    # weights follow numpy promotion: f32 * python int stays f32, * int64 array -> f64
    x = np.float32([0.1, 0.7])
    assert np.array_equal(o.quantize(x, 3), ((x * 3) * 2**18).astype(np.int64).astype(np.uint64))
    w = np.array([3, 3])
    assert np.array_equal(o.quantize(x, w), ((x * w) * 2**18).astype(np.int64).astype(np.uint64))


def test_golden_vectors_reproduce(golden_dir):
    g = np.load(os.path.join(golden_dir, "secagg_small.npz"))
    seeds = [int(h, 16) for h in g["stream_seeds_hex"]]
    for i, s in enumerate(seeds):
        st, inc = o.pcg64_state(s)
        assert hex(st) == g["stream_state_hex"][i] and hex(inc) == g["stream_inc_hex"][i]
        for j, off in enumerate(g["stream_offsets"]):
            assert np.array_equal(o.mask_stream(s, 16, int(off)), g["streams"][i, j])
    assert np.array_equal(o.quantize(g["q_in_f32"]), g["q_out_f32"])
    assert np.array_equal(o.quantize(g["q_in_f64"]), g["q_out_f64"])
    xs = list(g["round_x"])
    dec, s, masked = o.secure_sum(xs, ["alice", "bob", "carol"], offset=int(g["round_offset"]))
    assert np.array_equal(np.stack(masked), g["round_masked"])
    assert np.array_equal(s, g["round_sum"])
    assert np.array_equal(dec, g["round_decoded"])
    assert [o.digest(m) for m in masked] == [int(v) for v in g["round_digests"]]
    tol = 3 * 2.0**-18
    assert np.abs(dec - np.sum(np.stack(xs).astype(np.float64), axis=0)).max() < tol


def test_single_party_has_no_masks():
    x = np.float32([1.25, -2.5])
    dec, s, masked = o.secure_sum([x], ["alice"])
    assert np.array_equal(masked[0], o.quantize(x))
    assert np.array_equal(dec, x.astype(np.float64))


def test_numpy_scalar_weights_follow_numpy_1_23_value_based_casting():
    """The reference pins numpy 1.23.5 (uv.lock:1189-1190): a numpy-scalar
    weight does not widen float32 data (numpy 2's NEP 50 would).  Oracle and
    plugin agree on the arithmetic type; python scalars and array weights
    promote as before."""
    import numpy as np

    from sfl_amd.security.aggregation.secure_aggregator import _compute_dtype

    f32, f64, i64 = np.dtype(np.float32), np.dtype(np.float64), np.dtype(np.int64)
    cases = [(f32, np.float64(3.0), f32), (f32, np.int64(5), f32), (f32, np.float64(1e300), f64),
             (f32, 3, f32), (f32, 2.5, f32), (f32, np.array([1, 2], dtype=np.int64), f64),
             (f64, np.float32(2), f64), (i64, np.int64(3), i64), (i64, np.float64(0.5), f64),
             (f32, np.array(7.0), f32)]
    for dt, w, want in cases:
        if isinstance(w, np.generic) or (isinstance(w, np.ndarray) and w.ndim == 0):
            assert o.legacy_scalar_dtype(dt, w) == want, (dt, w)
        assert _compute_dtype(dt, w, 18) == want, (dt, w)
    x = np.float32([0.1, -0.3, 1.7])
    # float32 arithmetic with the weight rounded to float32, like numpy 1.23.5
    exp = np.trunc((x * np.float32(3.3)) * np.float32(1 << 18)).astype(np.int64).astype(np.uint64)
    assert np.array_equal(o.quantize(x, np.float64(3.3)), exp)
