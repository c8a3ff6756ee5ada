#!/usr/bin/env python3
"""Wave timeline of one fused masking launch (tuning only).  Needs the
SA_TIMING variant of the library:

    make -C sfl_amd/csrc VARIANT=_ts EXTRA=-DSA_TIMING
    SFL_SA_LIB=sfl_amd/lib/libsfl_sa_ts.so python tools/wave_timeline.py

Every wave's lane 0 records s_memrealtime (100 MHz) at entry, after the
prologue, after its first tile, after its last tile and at the end
(sa_clients_impl.h, SA_TIMING).  Prints where a launch's time goes beyond the
steady-state tile loop: dispatch ramp, prologue, first-tile warm-up, tail
imbalance, epilogue.
"""
import argparse
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# timing tool: may load a tuning variant (SFL_SA_LIB) that the product loader refuses
os.environ.setdefault("SFL_SA_ALLOW_TUNING_BUILD", "1")
sys.path.insert(0, ROOT)
TICK_US = 0.01  # s_memrealtime: 100 MHz


def pct(a, ps=(0, 1, 10, 50, 90, 99, 100)):
    return {f"p{p}": round(float(np.percentile(a, p)), 2) for p in ps}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--elems", type=int, default=100_000_000)
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--launches", type=int, default=3)
    args = ap.parse_args()
    import torch

    from bench import pair_seed
    from sfl_amd import _lib
    from sfl_amd import kernels as K
    from sfl_amd.parallel_sum import plan_generators, plan_rank

    _lib.lib()  # loads the library (SFL_SA_LIB) and checks the ABI
    raw = ctypes.CDLL(_lib.LIB_PATH)
    tl = raw.sa_debug_timeline
    tl.argtypes = [ctypes.c_void_p, ctypes.c_int]
    tl.restype = ctypes.c_int
    dev = torch.device("cuda", 0)
    N = args.elems
    names = [f"client{c}" for c in range(args.clients)]
    plan = plan_rank(names, 1, 0)
    xs = [torch.randn(N, device=dev) * 1e-2 for _ in plan.clients]
    pg, ps, cross = plan_generators(plan, pair_seed)
    s = torch.empty(N, dtype=torch.int64, device=dev)

    def run():
        K.fused_clients(xs, [1.0] * len(plan.clients), pg, ps, cross, plan.n_cross, s)

    for _ in range(3):
        run()
    torch.cuda.synchronize()
    buf = np.zeros((16384, 8), dtype=np.uint64)
    out = {"lib": _lib.LIB_PATH, "elems": N, "clients": args.clients, "launches": []}
    for _ in range(args.launches):
        assert tl(None, 1) == 0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        run()
        e1.record()
        torch.cuda.synchronize()
        assert tl(buf.ctypes.data, 0) == 0
        w = buf[buf[:, 0] != 0].astype(np.int64)
        t0 = w[:, 0].min()
        rel = (w[:, :5] - t0) * TICK_US
        tiles = w[:, 5]
        steady = (rel[:, 3] - rel[:, 2]) / np.maximum(tiles - 1, 1)
        first = rel[:, 2] - rel[:, 1]
        xcc = w[:, 7] & 0xF
        hw = w[:, 6]
        cu = (hw >> 8) & 0xF
        se = (hw >> 13) & 0x7
        per_xcc = {}
        for x in np.unique(xcc):
            m = xcc == x
            per_xcc[int(x)] = {"waves": int(m.sum()), "start_p50": round(float(np.median(rel[m, 0])), 2),
                               "loop_end_max": round(float(rel[m, 3].max()), 2),
                               "end_max": round(float(rel[m, 4].max()), 2)}
        simd_key = ((xcc * 8 + se) * 16 + cu) * 4 + ((hw >> 4) & 3)
        simd_end, simd_diff, older_fast, pairs = {}, {}, 0, 0
        for k in np.unique(simd_key):
            m = np.nonzero(simd_key == k)[0]
            e = rel[m, 3]
            simd_end[k], simd_diff[k] = e.max(), e.max() - e.min()
            if len(m) == 2:  # older wave: earlier start, then lower slot
                o, y = sorted(m, key=lambda j: (w[j, 0], hw[j] & 0xF))
                older_fast += int(steady[o] < steady[y])
                pairs += 1
        rec = {
            "event_ms": round(e0.elapsed_time(e1), 4),
            "waves": int(len(w)),
            "span_us": round(float(rel[:, 4].max()), 2),
            "tiles_per_wave": pct(tiles, (0, 50, 100)),
            "start_us": pct(rel[:, 0]),
            "prologue_us": pct(rel[:, 1] - rel[:, 0]),
            "first_tile_us": pct(first),
            "steady_tile_us": pct(steady),
            "loop_end_us": pct(rel[:, 3]),
            "epilogue_us": pct(rel[:, 4] - rel[:, 3]),
            "end_us": pct(rel[:, 4]),
            "simd_end_us": pct(list(simd_end.values())),
            "simd_wave_end_spread_us": pct(list(simd_diff.values())),
            "older_wave_faster_frac": round(older_fast / pairs, 3) if pairs else None,
            "ideal_us": round(float(np.median(steady) * tiles.max()), 2),
            "n_cu_se": int(len(np.unique(xcc * 1000 + se * 100 + cu))),
            "per_xcc": per_xcc,
        }
        out["launches"].append(rec)
        print(json.dumps(rec), flush=True)
    path = os.path.join(ROOT, "gpurun_out", "wave_timeline.json")
    os.makedirs(os.path.dirname(path), exist_ok=True)
    with open(path, "w") as f:
        json.dump(out, f, indent=1)
    np.save(os.path.join(ROOT, "gpurun_out", "wave_timeline_last.npy"), buf)


if __name__ == "__main__":
    main()
