"""The full-size GPU tests pin a 100M-element launch to the oracle through
windows (tests/oracle_windows.py).  On the CPU: the window restatement agrees
with the oracle's whole-vector computation and catches a single wrong element."""
import numpy as np
import pytest
import torch

from oracle import secagg as o
from oracle_windows import check_partial_sum_windows, window_starts


def test_windows_cover_ends_middle_and_joins():
    st = window_starts(1_000_000, 4096, joins=[125_000, 250_000], k_random=5)
    assert st[0] == 0 and st[-1] == 1_000_000 - 4096
    assert any(s < 125_000 < s + 4096 for s in st) and any(s < 250_000 < s + 4096 for s in st)
    assert len(st) >= 8


@pytest.mark.parametrize("clients", [[0, 1, 2, 3], [1], [0, 2]])
def test_window_check_matches_whole_vector_oracle(clients):
    C, n, off = 4, 40_000, 10**9 + 7
    names = [f"client{c}" for c in range(C)]
    seeds = o.seeds_for(names)
    rng = np.random.default_rng(len(clients))
    xs = [(rng.standard_normal(n) * 1e-2).astype(np.float32) for _ in range(C)]
    masked = o.secure_masked(xs, names, seeds=seeds, offset=off)
    part = o.server_sum([masked[c] for c in clients]).view(np.int64).copy()
    tx = [torch.from_numpy(x) for x in xs]
    assert check_partial_sum_windows(torch.from_numpy(part), tx, clients, names, seeds, off,
                                     joins=[n // 3]) >= 8 * 4096
    part[n - 1] ^= 1
    with pytest.raises(AssertionError, match=f"first at {n - 1}"):
        check_partial_sum_windows(torch.from_numpy(part), tx, clients, names, seeds, off)
