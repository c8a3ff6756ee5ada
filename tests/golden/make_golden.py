"""Generate the golden fixtures under tests/golden/ (committed).

* notebook_kat.json — the known-answer test printed in the reference's
  docs/developer/algorithm/secure_aggregation.ipynb (cells 7, 17, 18): the two
  parties' inputs (printed to 8 digits), the SecureAggregator's secure sum and
  secure average outputs, and the plain float sum.  Pure data, transcribed.
* aggregator_contract.json — inputs/expected values of the AggregatorBase
  contract (tests/security/aggregation/test_aggregator_base.py:21-160).
* secagg_small.npz — vectors from the numpy oracle (oracle/secagg.py, which
  calls numpy's own PCG64/Generator: the reference's arithmetic dependency):
  mask streams at offsets, quantize edge cases, and a 3-party masked round.

Run from the repo root:  python tests/golden/make_golden.py
"""
import json
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))
from oracle import secagg as o  # noqa: E402


def kat():
    return {
        "source": "docs/developer/algorithm/secure_aggregation.ipynb cells 7, 17, 18",
        "fxp_bits": 18,
        "parties": ["alice", "bob"],
        "arr0": [[0.53867365, 0.69040348, 0.42628929], [0.76128941, 0.5444343, 0.7680543]],
        "arr1": [[0.74303296, 0.7274792, 0.47244091], [0.88295957, 0.80091356, 0.82681861]],
        "plain_sum": [[1.28170662, 1.41788268, 0.8987302], [1.64424898, 1.34534786, 1.59487291]],
        "secure_sum": [[1.28170395, 1.41788101, 0.89872742], [1.64424515, 1.34534454, 1.59486771]],
        "secure_average": [[0.64085197, 0.70894051, 0.44936371], [0.82212257, 0.67267227, 0.79743385]],
        "note": "inputs are printed to 8 digits, so trunc-quantized re-runs match to ~5e-9",
    }


def contract():
    return {
        "source": "tests/security/aggregation/test_aggregator_base.py:21-160",
        "sum_single": {"a": [[1.0, 2.0, 3], [4.0, 5.0, 6.0]], "b": [[11.0, 12.0, 13.0], [14, 15.0, 16.0]],
                       "expect": [[12.0, 14.0, 16.0], [18.0, 20.0, 22.0]], "decimal": 5},
        "sum_list": {"a": [[[1, 2, 3], [4, 5, 6]], [[21, 22, 23], [24, 25, 26]]],
                     "b": [[[11, 12, 13], [14, 15, 16]], [[31, 32, 33], [34, 35, 36]]],
                     "expect": [[[12, 14, 16], [18, 20, 22]], [[52, 54, 56], [58, 60, 62]]], "decimal": 5},
        "avg_single": {"a": [[1.0, 2.0, 3.0], [4.0, 5.0, 6.0]], "b": [[11.0, 12.0, 13.0], [14.0, 15.0, 16.0]],
                       "expect": [[6.0, 7.0, 8.0], [9.0, 10.0, 11.0]], "decimal": 5},
        "avg_list": {"a": [[[1, 2, 3], [4, 5, 6]], [[21, 22, 23], [24, 25, 26]]],
                     "b": [[[11, 12, 13], [14, 15, 16]], [[31, 32, 33], [34, 35, 36]]],
                     "expect": [[[6, 7, 8], [9, 10, 11]], [[26, 27, 28], [29, 30, 31]]], "decimal": 5},
        "avg_weights": {"a": [[1, 2, 3], [4, 5, 6]], "b": [[11, 12, 13], [14, 15, 16]], "weights": [2, 3],
                        "expect": [[7, 8, 9], [10, 11, 12]], "decimal": 4},
        "avg_list_weights": {"a": [[[1, 2, 3], [4, 5, 6]], [[21, 22, 23], [24, 25, 26]]],
                             "b": [[[11, 12, 13], [14, 15, 16]], [[31, 32, 33], [34, 35, 36]]],
                             "weights": [2, 3],
                             "expect": [[[7, 8, 9], [10, 11, 12]], [[27, 28, 29], [30, 31, 32]]], "decimal": 4},
        "avg_same_shape_weights": {"a": [[1, 2, 3]], "b": [[11, 12, 13]],
                                   "weights": [[[5, 7, 2]], [[5, 3, 8]]], "decimal": 4},
    }


def small():
    out = {}
    seeds = [0, 1, o.pair_seed(0, 1), o.pair_seed(2, 5), 2**64 + 17, 2**127 + 3]
    out["stream_seeds_hex"] = np.array([hex(s) for s in seeds])
    offs = [0, 1, 1000, 123457]
    out["stream_offsets"] = np.array(offs, dtype=np.int64)
    out["streams"] = np.stack([np.stack([o.mask_stream(s, 16, off) for off in offs]) for s in seeds])
    st = [o.pcg64_state(s) for s in seeds]
    out["stream_state_hex"] = np.array([hex(a) for a, _ in st])
    out["stream_inc_hex"] = np.array([hex(b) for _, b in st])
    # quantize edge cases (float32 and float64), fxp 18
    e32 = np.array([0.0, -0.0, 2.0**-18, -2.0**-18, 2.0**-19, -2.0**-19, 1.5 * 2.0**-18, -1.5 * 2.0**-18,
                    1.0, -1.0, 3.999999, -3.999999, 1e-3, -1e-3, 12345.678, -12345.678, 2.0**44, -2.0**44,
                    2.0**45, -2.0**45, 3e38, -3e38, np.inf, -np.inf, np.nan], dtype=np.float32)
    out["q_in_f32"] = e32
    out["q_out_f32"] = o.quantize(e32, None, 18)
    e64 = e32.astype(np.float64)
    e64[16:20] = [2.0**44 + 0.5, -(2.0**44 + 0.5), 2.0**45, -2.0**45]
    out["q_in_f64"] = e64
    out["q_out_f64"] = o.quantize(e64, None, 18)
    # a 3-party round, float32, n = 37 (ragged), offset 5 (second round)
    rng = np.random.default_rng(7)
    xs = [(rng.standard_normal(37) * 3).astype(np.float32) for _ in range(3)]
    names = ["alice", "bob", "carol"]
    dec, s, masked = o.secure_sum(xs, names, offset=5)
    out["round_x"] = np.stack(xs)
    out["round_masked"] = np.stack(masked)
    out["round_sum"] = s
    out["round_decoded"] = dec
    out["round_offset"] = np.array(5)
    out["round_digests"] = np.array([o.digest(m) for m in masked], dtype=np.uint64)
    return out


if __name__ == "__main__":
    with open(os.path.join(HERE, "notebook_kat.json"), "w") as f:
        json.dump(kat(), f, indent=1)
    with open(os.path.join(HERE, "aggregator_contract.json"), "w") as f:
        json.dump(contract(), f, indent=1)
    np.savez(os.path.join(HERE, "secagg_small.npz"), **small())
    print("golden fixtures written")
