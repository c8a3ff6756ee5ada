"""DP pre-step oracle (host, no GPU): Philox4x32-10 known-answer vectors
(Random123 kat_vectors, philox4x32 with 10 rounds) and the clip formula of
sfl/security/privacy/mechanism/mechanism_fl.py restated in numpy."""
import numpy as np
import pytest

from oracle import dp as D

KAT = [
    ((0, 0, 0, 0), (0, 0), (0x6627E8D5, 0xE169C58D, 0xBC57AC4C, 0x9B00DBD8)),
    ((0xFFFFFFFF,) * 4, (0xFFFFFFFF, 0xFFFFFFFF), (0x408F276D, 0x41C83B0E, 0xA20BC7C6, 0x6D5451FD)),
    ((0x243F6A88, 0x85A308D3, 0x13198A2E, 0x03707344), (0xA4093822, 0x299F31D0),
     (0xD16CFE09, 0x94FDCCEB, 0x5001E420, 0x24126EA1)),
]


@pytest.mark.parametrize("ctr,key,exp", KAT)
def test_philox_known_answers(ctr, key, exp):
    out = D.philox4x32_10(np.array([ctr], dtype=np.uint32), key)
    assert tuple(int(v) for v in out[0]) == exp


def test_gauss_stream_layout_and_moments():
    z = D.gauss(123, 0, 400_000)
    assert abs(z.mean()) < 5e-3 and abs(z.std() - 1) < 5e-3
    # element e is normal (e & 3) of block e >> 2, whatever the starting counter
    assert np.array_equal(D.gauss(123, 8, 10), z[8:18])
    assert np.array_equal(D.gauss(123, 12, 3), z[12:15])


def test_clip_formula_matches_reference_expression():
    """GaussianModelDP without noise (noise_multiplier = 0) is the reference's
    `inputs[i] * min(1, clip / global_norm)` in float32."""
    rng = np.random.default_rng(0)
    layers = [rng.standard_normal((7, 5)).astype(np.float32), rng.standard_normal(11).astype(np.float32)]
    out = D.gaussian_model_dp(layers, noise_multiplier=0.0, num_updates=4, l2_norm_clip=0.5)
    norm = np.sqrt(sum(np.linalg.norm(a.astype(np.float64)) ** 2 for a in layers))
    scale = np.float32(min(1.0, 0.5 / np.float32(norm)))
    for a, b in zip(layers, out):
        assert b.dtype == np.float32
        assert np.array_equal(b, a * scale)
    # per-layer clipping: min(1, clip / sqrt(norm_layer * norm_all))
    out = D.gaussian_model_dp(layers, 0.0, 4, 0.5, is_clip_each_layer=True)
    for a, b in zip(layers, out):
        nl = np.float32(np.linalg.norm(a.astype(np.float64)))
        s = np.float32(min(1.0, np.float32(0.5) / np.sqrt(nl * np.float32(norm))))
        assert np.allclose(b, a * s, rtol=2e-7, atol=0)


@pytest.mark.parametrize("each_layer", [False, True])
def test_clip_restatement_vs_numpy_reference_arithmetic(each_layer):
    """oracle.dp's clip (the device's arithmetic) against mechanism_fl.py:
    71-108,132-135 evaluated by numpy itself (noise 0): equal up to the
    reference's float32 BLAS dot error, measured here, plus 4 ulps; the
    float32 structure of the norm (per-layer float32 norm, ** 2, float32
    sum) is what the oracle restates."""
    rng = np.random.default_rng(4)
    layers = [(rng.standard_normal(s) * 0.05).astype(np.float32) for s in ((64, 50), (50,), (50, 3), (3,))]

    def gnorm(arrs):
        return np.sqrt(sum([np.linalg.norm(a) ** 2 for a in arrs]))

    norm_all = gnorm(layers)
    if each_layer:
        ref = [a * min(1, 0.5 / np.sqrt(gnorm([a]) * norm_all)) for a in layers]
    else:
        ref = [a * min(1, 0.5 / norm_all) for a in layers]
    got = D.gaussian_model_dp(layers, 0.0, 8, 0.5, is_clip_each_layer=each_layer)
    exact = [np.sqrt(np.sum(a.astype(np.float64) ** 2)) for a in layers]
    rel = max(abs(float(np.linalg.norm(a)) - e) / e for a, e in zip(layers, exact))
    for g, r in zip(got, ref):
        np.testing.assert_allclose(g, r, rtol=2 * rel + 4 * 2.0**-24, atol=0)
    # the float32 structure: the squared global norm is a float32 sum of float32 squares
    t = np.float32(0)
    for a in layers:
        t = t + D.layer_sq_norm(a)
        assert t.dtype == np.float32
    assert D.global_sq(layers) == t
