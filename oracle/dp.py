"""CPU restatement of the DP pre-step -- TEST INFRASTRUCTURE ONLY (the
checker for tests/ and bench.py's baseline; the product path never imports
it).

* GaussianModelDP clip formula: sfl/security/privacy/mechanism/mechanism_fl.py
  :71 (global norm), :81-84 (per-layer scale), :104-108 (global scale),
  :112-127 (noise / num_updates, np.add), :132-135 (global_norm: float32
  np.linalg.norm per layer, ** 2, python sum, np.sqrt), with numpy 1.23.5's
  scalar promotion (the reference's pin, uv.lock:1189-1190): an operation
  between two scalars promotes by type alone (no value-based casting), so a
  python int / float meets a float32 scalar as int64 / float64 -- ``** 2``,
  the python sum, ``np.sqrt`` of it and ``clip / norm`` are all float64;
  value-based casting applies only with an array (the float32 array times
  the float64 scale stays float32).  One deviation:
  the layer's dot is the exact float64 sum rounded once to float32, where
  the reference's BLAS sdot accumulates in float32 in its own order
  (|difference| <= n * 2^-24 of the dot in the worst case).
* Philox4x32-10: Salmon, Moraes, Dror, Shaw, "Parallel random numbers: as
  easy as 1, 2, 3" (SC'11), Random123 constants; pinned by the published
  known-answer vectors in tests/test_dp_oracle.py.
* Box-Muller of the kernels' sa_philox.h (u1 = ((r >> 8) + 1) / 2^24,
  u2 = (r >> 8) / 2^24); numpy's transcendental functions round differently
  from the device's, so noise compares within a tolerance.
"""

import numpy as np

M0, M1 = np.uint64(0xD2511F53), np.uint64(0xCD9E8D57)
W0, W1 = 0x9E3779B9, 0xBB67AE85
MASK32 = np.uint64(0xFFFFFFFF)


def philox4x32_10(ctr: np.ndarray, key) -> np.ndarray:
    """ctr: (n, 4) uint32 counters, key: (k0, k1) -> (n, 4) uint32."""
    c = [ctr[:, j].astype(np.uint64) for j in range(4)]
    k0, k1 = int(key[0]) & 0xFFFFFFFF, int(key[1]) & 0xFFFFFFFF
    for _ in range(10):
        p0 = M0 * c[0]
        p1 = M1 * c[2]
        n0 = (p1 >> np.uint64(32)) ^ c[1] ^ np.uint64(k0)
        n2 = (p0 >> np.uint64(32)) ^ c[3] ^ np.uint64(k1)
        c = [n0 & MASK32, p1 & MASK32, n2 & MASK32, p0 & MASK32]
        k0 = (k0 + W0) & 0xFFFFFFFF
        k1 = (k1 + W1) & 0xFFFFFFFF
    return np.stack(c, axis=1).astype(np.uint32)


def gauss(key: int, counter0: int, n: int) -> np.ndarray:
    """Standard normals of elements counter0 .. counter0+n-1 (float32)."""
    b0, b1 = counter0 // 4, (counter0 + n + 3) // 4
    blk = np.arange(b0, b1, dtype=np.uint64)
    ctr = np.zeros((blk.size, 4), dtype=np.uint32)
    ctr[:, 0] = (blk & MASK32).astype(np.uint32)
    ctr[:, 1] = (blk >> np.uint64(32)).astype(np.uint32)
    r = philox4x32_10(ctr, (key & 0xFFFFFFFF, key >> 32))
    z = np.empty((blk.size, 4), dtype=np.float32)
    for j in range(2):
        u1 = ((r[:, 2 * j] >> 8).astype(np.float32) + np.float32(1)) * np.float32(2.0**-24)
        u2 = (r[:, 2 * j + 1] >> 8).astype(np.float32) * np.float32(2.0**-24)
        rad = np.sqrt(np.float32(-2) * np.log(u1))
        ang = np.float32(2) * u2
        z[:, 2 * j] = rad * np.cos(np.pi * ang.astype(np.float64)).astype(np.float32)
        z[:, 2 * j + 1] = rad * np.sin(np.pi * ang.astype(np.float64)).astype(np.float32)
    off = counter0 - b0 * 4
    return z.reshape(-1)[off:off + n]


def layer_norm32(a) -> np.float32:
    """``np.linalg.norm(a)`` of a float32 array (numpy 1.23.5: ``sqrt(x.dot(x))``
    in float32) -- the dot here the exact float64 sum rounded once (the
    reference's BLAS sdot adds in float32 in its own order)."""
    dot = np.float32(np.sum(np.asarray(a, dtype=np.float64).reshape(-1) ** 2))
    return np.sqrt(dot, dtype=np.float32)


def layer_sq_norm(a) -> np.float64:
    """One layer's ``np.linalg.norm(a) ** 2`` (mechanism_fl.py:133) under numpy
    1.23.5: the float32 norm ``** 2`` (a python int) is a scalar-scalar
    operation, promoted to float64 -- the exact square."""
    n = np.float64(layer_norm32(a))
    return n * n


def global_sq(inputs) -> np.float64:
    """``sum([np.linalg.norm(i) ** 2 for i in inputs])``: python's sum from 0
    over the float64 squares, in order (mechanism_fl.py:133)."""
    t = np.float64(0)
    for a in inputs:
        t = t + layer_sq_norm(a)
    return t


def clip_scale(sumsq, clip: float, sumsq_layer=None) -> np.float32:
    """min(1, clip / norm) as mechanism_fl.py:71-84,104-108 computes it under
    numpy 1.23.5, all in float64 scalars: norm_all = np.sqrt(sumsq) (float64,
    ``global_norm``); per layer the denominator np.sqrt(layer_norm *
    norm_all) with layer_norm = np.sqrt(layer square) (= the float32 norm,
    exactly); the python-float clip divided in float64.  ``inputs[i] *
    scale`` then rounds the float64 scale to float32 (value-based casting: an
    array times a scalar keeps the array's float32)."""
    norm_all = np.sqrt(np.float64(sumsq))
    denom = norm_all
    if sumsq_layer is not None:
        denom = np.sqrt(np.sqrt(np.float64(sumsq_layer)) * norm_all)
    with np.errstate(divide="ignore", invalid="ignore"):
        r = np.float64(float(clip)) / denom
    return np.float32(r) if r < 1.0 else np.float32(1)


def perturb(x: np.ndarray, scale, z: np.ndarray, sigma: float, num_updates: float) -> np.ndarray:
    """float32 x * scale + (z * sigma) / num_updates (reference op order)."""
    x = np.asarray(x, dtype=np.float32)
    noise = z.astype(np.float32) * np.float32(sigma)
    return x * np.float32(scale) + noise / np.float32(num_updates)


def gaussian_model_dp(inputs, noise_multiplier, num_updates, l2_norm_clip=1.0, key=0, counter0=0,
                      is_clip_each_layer=False):
    """Restated GaussianModelDP.__call__ with this build's noise stream."""
    sigma = noise_multiplier * l2_norm_clip * l2_norm_clip
    total = global_sq(inputs)
    out, ctr = [], counter0
    for a in inputs:
        a = np.asarray(a, dtype=np.float32)
        lay = layer_sq_norm(a) if is_clip_each_layer else None
        s = clip_scale(total, l2_norm_clip, lay)
        z = gauss(key, ctr, a.size)
        out.append(perturb(a.reshape(-1), s, z, sigma, num_updates).reshape(a.shape))
        ctr += -(-a.size // 4) * 4
    return out
