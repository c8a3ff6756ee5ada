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


def _legacy_numpy_clip(inputs, clip, each_layer):
    """mechanism_fl.py:71-108,132-135 with noise_multiplier = 0, evaluated BY
    HAND with numpy 1.23.5's promotion written out (this image's numpy 2
    follows NEP 50 and cannot run it):

    * ``np.linalg.norm(a)`` of a float32 array: ``sqrt(a.dot(a))`` in float32
      (the dot taken exactly here and rounded once; BLAS order aside);
    * ``norm ** 2``: float32 scalar with a python int -- scalar-scalar, no
      value-based casting in 1.x: ``promote_types(float32, int64)`` = float64;
    * ``sum(...)`` from the python int 0: float64 adds in order;
    * ``np.sqrt`` of a float64 scalar: float64; ``clip / norm`` and
      ``np.sqrt(gn * norm_all)``: float64;
    * ``inputs[i] * scale``: array with a scalar -- value-based casting keeps
      float32, the scalar rounded to float32 first."""
    def norm32(a):
        x = a.astype(np.float64).ravel()
        return np.sqrt(np.float32(np.dot(x, x)), dtype=np.float32)

    def global_norm(arrs):
        total = 0
        for a in arrs:
            total = total + np.float64(norm32(a)) * np.float64(norm32(a))
        return np.sqrt(np.float64(total))

    norm_all = global_norm(inputs)
    out = []
    for a in inputs:
        if each_layer:
            r = np.float64(clip) / np.sqrt(global_norm([a]) * norm_all)
        else:
            r = np.float64(clip) / norm_all
        scale = r if r < 1 else 1
        out.append(a * np.float32(scale))
    return out


def _float32_model_clip(inputs, clip, each_layer):
    """The round-4 model (every scalar float32 but the division) -- what a
    regression to it would compute; used to show the test can tell them apart."""
    def norm32(a):
        x = a.astype(np.float64).ravel()
        return np.sqrt(np.float32(np.dot(x, x)), dtype=np.float32)

    t = np.float32(0)
    for a in inputs:
        t = np.float32(t + np.float32(norm32(a) * norm32(a)))
    norm_all = np.sqrt(t, dtype=np.float32)
    out = []
    for a in inputs:
        d = np.sqrt(np.float32(norm32(a) * norm_all), dtype=np.float32) if each_layer else norm_all
        r = np.float64(np.float32(clip)) / np.float64(d)
        out.append(a * (np.float32(r) if r < 1 else np.float32(1)))
    return out


@pytest.mark.parametrize("each_layer", [False, True])
def test_clip_follows_numpy_1_23_scalar_promotion(each_layer):
    """the oracle's clip (the device's arithmetic) equals, BIT FOR
    BIT, the reference formula under numpy 1.23.5's promotion written out by
    hand (exact dots, so the BLAS order does not enter); and that check can
    tell the float64-scalar model from the float32 one (inputs where they
    differ exist and are among the cases)."""
    rng = np.random.default_rng(21)
    differ = 0
    for trial in range(40):
        shapes = [tuple(rng.integers(1, 40, size=int(rng.integers(1, 3)))) for _ in range(int(rng.integers(1, 5)))]
        layers = [(rng.standard_normal(s) * rng.uniform(0.01, 3)).astype(np.float32) for s in shapes]
        clip = float(rng.choice([0.1, 0.3, 0.5, 1.0, 2.5]))
        got = D.gaussian_model_dp(layers, 0.0, 4, clip, is_clip_each_layer=each_layer)
        want = _legacy_numpy_clip(layers, clip, each_layer)
        for g, w in zip(got, want):
            assert g.dtype == np.float32 and np.array_equal(g, w), trial
        old = _float32_model_clip(layers, clip, each_layer)
        differ += any(not np.array_equal(g, o) for g, o in zip(got, old))
    assert differ > 0


@pytest.mark.parametrize("each_layer", [False, True])
def test_clip_restatement_vs_numpy_reference_arithmetic(each_layer):
    """oracle.dp's clip (the device's arithmetic) against mechanism_fl.py:
    71-108,132-135 evaluated by this image's numpy 2 itself (noise 0; NEP 50,
    so every scalar float32): equal up to the reference's float32 BLAS dot
    error, measured here, plus 4 ulps -- a sanity check only: parity with
    numpy 1.23.5's float64 scalars is test_clip_follows_numpy_1_23_scalar_promotion."""
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
    # numpy 1.23.5's structure: float32 layer norms, float64 exact squares and sum
    t = 0
    for a in layers:
        n32 = D.layer_norm32(a)
        assert n32.dtype == np.float32 and D.layer_sq_norm(a) == np.float64(n32) ** 2
        t = t + D.layer_sq_norm(a)
        assert t.dtype == np.float64
    assert D.global_sq(layers) == t
