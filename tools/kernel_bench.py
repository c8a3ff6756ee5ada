#!/usr/bin/env python3
"""Kernel-level timing of the masking kernels for tuning (not the headline
bench).  Times sa_fused_clients for the per-rank shapes of C clients split
over W GPUs (rank 0's share, no RCCL) and the single-client sa_mask, with
hipEvents, interleaving configurations over several rounds in one process.

usage: python tools/kernel_bench.py [--elems N] [--rounds R] [--shapes 8:1,8:2,8:4,8:8]
Set SFL_SA_LIB to time a tuning variant of libsfl_sa.so.
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# timing tool: may load a tuning variant (SFL_SA_LIB) that the product loader refuses
os.environ.setdefault("SFL_SA_ALLOW_TUNING_BUILD", "1")
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--elems", type=int, default=100_000_000)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--shapes", default="8:1,8:2,8:4,8:8", help="C:W pairs")
    ap.add_argument("--bipartite", action="store_true",
                    help="also time one sa_fused_bipartite launch (16 cross pairs of two quads, masks only, "
                         "accumulating into the sum: 16 B of HBM traffic per element)")
    ap.add_argument("--fallback", action="store_true",
                    help="also time the per-client path (two sa_mask passes per client, accumulating into the "
                         "sum) for every shape beyond one fused launch, interleaved with its multi-launch schedule")
    ap.add_argument("--calib", type=int, default=0,
                    help="also launch sa_sum_u64 over this many u64 inputs (known bytes, for PMC calibration)")
    args = ap.parse_args()
    import torch

    from bench import pair_seed
    from sfl_amd import _lib
    from sfl_amd import kernels as K
    from sfl_amd.parallel_sum import plan_generators, plan_rank

    _lib.lib()
    dev = torch.device("cuda", 0)
    N = args.elems
    shapes = [tuple(int(v) for v in s.split(":")) for s in args.shapes.split(",")]
    cases = []
    for C, W in shapes:
        names = [f"client{c}" for c in range(C)]
        plan = plan_rank(names, W, 0)
        xs = [torch.randn(N, device=dev) * 1e-2 for _ in plan.clients]
        pg, ps, cross = plan_generators(plan, pair_seed)
        s = torch.empty(N, dtype=torch.int64, device=dev)
        cases.append(dict(C=C, W=W, L=len(plan.clients), plan=plan, xs=xs, pg=pg, ps=ps, cross=cross, s=s,
                          times=[], path="fused"))
        if args.fallback and len(plan.pairs) + len(plan.cross) > 32:
            cases.append(dict(cases[-1], times=[], path="per-client fallback"))
    for _ in range(args.rounds):
        for cs in cases:
            def run():
                fn = K.fused_clients if cs["path"] == "fused" else K._fused_fallback
                if fn is K.fused_clients:
                    fn(cs["xs"], [1.0] * cs["L"], cs["pg"], cs["ps"], cs["cross"], cs["plan"].n_cross, cs["s"])
                else:
                    fn(cs["xs"], [1.0] * cs["L"], cs["pg"], cs["ps"], cs["cross"], cs["plan"].n_cross, cs["s"], 18,
                       False, None, None, None)
            run()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                run()
            e1.record()
            torch.cuda.synchronize()
            cs["times"].append(e0.elapsed_time(e1) / args.reps)
    bip = None
    if args.bipartite:
        import ctypes as C

        from sfl_amd import _lib as L

        clients = (L.LocalClient * 8)()
        for c in range(8):
            clients[c].x, clients[c].weight, clients[c].masked_out = None, 1.0, None
        gens = (L.PCG64 * 16)(*[L.pcg64_from_seed(pair_seed(p // 4, 4 + p % 4)) for p in range(16)])
        signs = (C.c_int8 * 16)(*([1] * 16))
        sb = torch.zeros(N, dtype=torch.int64, device=dev)

        def run_bip():
            L.check(L.lib().sa_fused_bipartite(clients, L.SA_F32, N, 18, gens, signs, C.c_void_p(sb.data_ptr()), 1,
                                               None, C.c_void_p(torch.cuda.current_stream().cuda_stream)), "bip")
        times = []
        for _ in range(args.rounds):
            run_bip()
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            for _ in range(args.reps):
                run_bip()
            e1.record()
            torch.cuda.synchronize()
            times.append(e0.elapsed_time(e1) / args.reps)
        t = sorted(times)[len(times) // 2]
        bip = {"kernel": "k_clients<float, float, 8, 0, 1> (sa_fused_bipartite)", "ms_median": t,
               "pair_draws_per_s": 16 * N / (t / 1e3), "hbm_GBps": 16 * N / (t / 1e3) / 1e9}
    if args.calib:
        ins = [torch.randint(0, 1 << 62, (N,), device=dev) for _ in range(args.calib)]
        so = torch.empty(N, dtype=torch.int64, device=dev)
        for _ in range(args.reps):
            K.sum_u64(ins, so)
        torch.cuda.synchronize()
        del ins
    out = []
    for cs in cases:
        t = sorted(cs["times"])
        ms = t[len(t) // 2]
        draws = (len(cs["plan"].pairs) + len(cs["plan"].cross)) * N
        out.append({"C": cs["C"], "W": cs["W"], "L": cs["L"], "path": cs["path"], "ms_median": ms, "ms_min": t[0],
                    "draws_per_s": draws / (ms / 1e3), "local_grad_elems_per_s": cs["L"] * N / (ms / 1e3),
                    "hbm_GBps": (4 * cs["L"] * N + 8 * N) / (ms / 1e3) / 1e9})
    res = {"lib": os.environ.get("SFL_SA_LIB", "default"), "elems": N, "cases": out}
    if bip:
        res["bipartite"] = bip
    print(json.dumps(res))


if __name__ == "__main__":
    main()
