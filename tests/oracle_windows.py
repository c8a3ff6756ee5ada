"""Oracle windows of a full-size masked sum (test helper).

A 100M-element launch is too big for the numpy oracle as a whole, but the
oracle can restate any contiguous window of it exactly: every pair stream is
jumped to the window's first element (``PCG64.advance``) and the window's
clients are quantized, masked and summed as the reference does.  Comparing
the device's own output at several windows (both ends, the middle, chunk
joins, random offsets) pins the launch the bench times to the oracle
directly, without going through another HIP path.
"""
from __future__ import annotations

import numpy as np
import torch

from oracle import secagg as o


def window_starts(n: int, w: int, joins=(), k_random: int = 5, seed: int = 0) -> list[int]:
    """Starts of windows of ``w`` elements: the start, the end, the middle,
    one straddling each chunk join, and ``k_random`` random offsets."""
    rng = np.random.default_rng(seed)
    starts = {0, max(0, n - w), max(0, n // 2 - w // 2)}
    starts |= {min(max(0, j - w // 2), max(0, n - w)) for j in joins}
    starts |= {int(s) for s in rng.integers(0, max(1, n - w), k_random)}
    return sorted(starts)


def check_partial_sum_windows(out: torch.Tensor, xs, clients, names, seeds, offset: int, w: int = 4096,
                              joins=(), k_random: int = 5, seed: int = 0) -> int:
    """Assert ``out`` (device uint64-as-int64, the masked sum of ``clients``'
    vectors ``xs[c]`` for every client c in ``clients``; the streams of every
    other client in ``names`` are the cross streams) equals the oracle on
    every window.  ``offset``: the round's stream position of element 0.
    Returns the number of element positions checked."""
    n = out.numel()
    checked = 0
    for s0 in window_starts(n, w, joins, k_random, seed):
        e = min(n, s0 + w)
        xh = [xs[c][s0:e].cpu().numpy() for c in clients]
        exp = np.zeros(e - s0, dtype=np.uint64)
        for c, x in zip(clients, xh):
            me = names[c]
            exp += o.mask_client(o.quantize(x), me, seeds[me], offset + s0)
        got = out[s0:e].cpu().numpy().view(np.uint64)
        bad = np.flatnonzero(got != exp)
        assert bad.size == 0, f"window [{s0}, {e}): {bad.size} elements differ, first at {s0 + int(bad[0])}"
        checked += e - s0
    return checked
