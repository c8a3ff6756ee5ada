#!/usr/bin/env python3
"""Headline benchmark (BASELINE.json `metric`):
    grad elems/s device-resident: 100M-float quantize+mask+sum, 8 clients

One step = one pass of the secure-aggregation hot path over one batch:
every client's 100M-float gradient (resident in HBM) is quantized to fixed
point (fxp 18), masked with its 7 pairwise PCG64 streams (mod 2^64) and
summed into the server's uint64 masked sum.  Rate = C*N / step time
(one "grad elem" = one fp32 element of one client).

N=1 (default): all 8 clients on one MI355X in ONE fused launch
(sa_fused_clients: L=8 local clients, 28 pair streams each expanded once).
N>1 (torchrun, one process per GPU): clients sharded in contiguous blocks
(8/N per GPU, config 3 at N=8); each rank runs one fused launch over its
clients (internal pairs + cross streams) and the uint64 partial sums are
reduced to rank 0 (the server) with ncclReduce over xGMI.  Total work is
fixed as N grows: "scaling": "strong".

Inputs: synthetic N(0, 0.01^2) fp32 gradients generated on the GPU
(torch.Generator seeded 20260116+c); pair seeds (0x5ECA66<<32)|(u<<16)|v as
in SURVEY.md §8(d).  Generator positions advance by N draws every step
(a new FL round each step), precomputed before the timed region.
"""

from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
if ROOT not in sys.path:
    sys.path.insert(0, ROOT)

HBM_PEAK_GBPS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
PCG_PEAK_DRAWS = 1.57e12        # measured PCG64 draw-loop ceiling (one-sided draws, 8 waves/SIMD),
                                # tools/microbench/draw_issue.hip "dual one7 E2", profiles/r01/draw_issue_microbench.txt


def pair_seed(u: int, v: int) -> int:
    a, b = (u, v) if u < v else (v, u)
    return (0x5ECA66 << 32) | (a << 16) | b


def cpu_baseline(C: int, fxp_bits: int, seconds: float) -> dict:
    """The numpy restatement (oracle/, kind "port") timed on this host on a
    bounded sample of the same workload: C clients, n_sample elements each."""
    import numpy as np

    from oracle import secagg as o

    names = [f"client{c}" for c in range(C)]
    seeds = {a: {b: pair_seed(i, j) for j, b in enumerate(names) if b != a} for i, a in enumerate(names)}

    def run(n):
        xs = [np.random.default_rng(20260116 + c).standard_normal(n, dtype=np.float32) * np.float32(1e-2)
              for c in range(C)]
        t0 = time.perf_counter()
        masked = o.secure_masked(xs, names, None, fxp_bits, seeds)
        o.server_sum(masked)
        return time.perf_counter() - t0

    t_cal = run(200_000)
    n = int(max(200_000, min(50_000_000, 200_000 * seconds / max(t_cal, 1e-6))))
    t = run(n)
    try:
        par = cpu_baseline_parallel(C, fxp_bits, n)
    except Exception as e:  # the single-threaded figure stands on its own
        par = {"error": repr(e)}
    try:
        cores = len(os.sched_getaffinity(0))
    except AttributeError:  # pragma: no cover
        cores = os.cpu_count()
    return {"value": C * n / t, "unit": "grad elems/s", "cores": 1, "kind": "port",
            "sample": f"{C} clients x {n} fp32 elems, oracle/secagg.py numpy (single-threaded), "
                      f"{t:.1f} s; host has {cores} cores available",
            "seconds": round(t, 3), "parallel": par}


def _cpu_party(args):
    """One client of the parallel CPU baseline: quantize + its C-1 pairwise
    masks (oracle/secagg.py numpy, single-threaded), the masked vector written
    into the shared server buffer.  Returns its timed region (monotonic)."""
    c, C, n, fxp_bits, shm_name = args
    from multiprocessing import shared_memory

    import numpy as np

    from oracle import secagg as o

    names = [f"client{i}" for i in range(C)]
    seeds = {b: pair_seed(c, j) for j, b in enumerate(names) if j != c}
    x = np.random.default_rng(20260116 + c).standard_normal(n, dtype=np.float32) * np.float32(1e-2)
    t0 = time.perf_counter()
    m = o.mask_client(o.quantize(x, None, fxp_bits), names[c], seeds)
    shm = shared_memory.SharedMemory(name=shm_name)
    np.ndarray((C, n), dtype=np.uint64, buffer=shm.buf)[c] = m
    t1 = time.perf_counter()
    del m
    shm.close()
    return t0, t1


def cpu_baseline_parallel(C: int, fxp_bits: int, n: int) -> dict:
    """SURVEY.md §8d's second CPU figure: one process per client (C cores, as
    the reference runs one party per process), masked vectors into shared
    memory, then the server sum.  Forked before this process touches the GPU."""
    import multiprocessing as mp
    from multiprocessing import shared_memory

    import numpy as np

    from oracle import secagg as o

    shm = shared_memory.SharedMemory(create=True, size=C * n * 8)
    try:
        with mp.get_context("fork").Pool(C) as pool:
            spans = pool.map(_cpu_party, [(c, C, n, fxp_bits, shm.name) for c in range(C)])
        masked = np.ndarray((C, n), dtype=np.uint64, buffer=shm.buf)
        t0 = time.perf_counter()
        o.server_sum(list(masked))
        t_sum = time.perf_counter() - t0
        del masked
    finally:
        shm.close()
        shm.unlink()
    t = max(b for _, b in spans) - min(a for a, _ in spans) + t_sum
    return {"value": C * n / t, "unit": "grad elems/s", "cores": C, "kind": "port",
            "sample": f"{C} client processes x {n} fp32 elems (oracle/secagg.py numpy), masked vectors in "
                      f"shared memory, then the server sum; {t:.1f} s",
            "seconds": round(t, 3)}


PMC_DIR = os.path.join(ROOT, "profiles", "r01")


def pmc_traffic(kernel: str) -> dict | None:
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (tools/gpu_profile.sh: separate FETCH_SIZE / WRITE_SIZE runs of
    tools/kernel_bench.py on this workload).  Units are KiB; gfx950 reports
    FETCH_SIZE at half the bytes of 16-B/lane streaming reads, so it is
    doubled (MI355X_MICROARCH.md, HBM); both corrections were checked on the
    k_sum_u64 calibration launch in the same runs (known bytes)."""
    import csv

    vals = {}
    for counter, fname, scale in (("FETCH_SIZE", "pmc_fetch_size.csv", 2.0), ("WRITE_SIZE", "pmc_write_size.csv", 1.0)):
        path = os.path.join(PMC_DIR, fname)
        if not os.path.exists(path):
            return None
        v = [float(r["Counter_Value"]) for r in csv.DictReader(open(path))
             if r["Kernel_Name"].startswith(kernel) and r["Counter_Name"] == counter]
        if not v:
            return None
        vals[counter] = scale * 1024.0 * sum(v) / len(v)
    return {"bytes": vals["FETCH_SIZE"] + vals["WRITE_SIZE"], "read": vals["FETCH_SIZE"], "write": vals["WRITE_SIZE"],
            "source": os.path.relpath(PMC_DIR, ROOT) + "/pmc_{fetch,write}_size.csv"}


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--elems", type=int, default=100_000_000)
    ap.add_argument("--fxp-bits", type=int, default=18)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=10.0, help="0 disables")
    ap.add_argument("--extra", action="store_true", help="also time the wire chain and H2D/D2H-inclusive rate")
    ap.add_argument("--dist", action="store_true",
                    help="run the multi-GPU code path (RCCL communicator, pipelined reduce) even at N=1 "
                         "(rehearsal of the N>1 path on one GPU under torchrun)")
    ap.add_argument("--chunks", type=int, default=None,
                    help="N>1: masking/reduce pipeline depth (default 8; 1 = reduce after the whole launch)")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    # CPU baseline first: its per-client worker processes are forked, which
    # must happen before this process initialises the GPU
    cpu = None
    if rank == 0 and world == 1 and args.cpu_baseline_seconds > 0:
        cpu = cpu_baseline(args.clients, args.fxp_bits, args.cpu_baseline_seconds)

    import torch
    import torch.distributed as dist

    from sfl_amd import _lib
    from sfl_amd import kernels as K
    from sfl_amd.parallel_sum import PipelinedMaskedSum, RcclComm, plan_generators, plan_rank

    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    torch.cuda.set_device(local_rank)
    dev = torch.device("cuda", local_rank)
    _lib.lib()
    comm = None
    multi = world > 1 or args.dist
    if multi:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        comm = RcclComm(rank, world, local_rank)

    C, N = args.clients, args.elems
    names = [f"client{c}" for c in range(C)]
    plan = plan_rank(names, world, rank)
    Lc = len(plan.clients)
    xs = []
    for c in plan.clients:
        g = torch.Generator(device=dev).manual_seed(20260116 + c)
        xs.append(torch.randn(N, generator=g, device=dev, dtype=torch.float32) * 1e-2)
    total_steps = args.warmup + args.steps
    chunks = args.chunks if args.chunks is not None else (8 if multi else 1)
    pipe = PipelinedMaskedSum(comm, dev, N, chunks)
    # every step is a new round: streams start i*N draws in, chunk j at +lo_j
    gens = [[plan_generators(plan, pair_seed, offset=i * N + lo) for lo, _ in pipe.bounds]
            for i in range(total_steps)]
    sum_buf = torch.empty(N, dtype=torch.int64, device=dev)
    recv = torch.empty(N, dtype=torch.int64, device=dev) if (rank == 0 and multi) else None
    digests = torch.zeros(Lc, dtype=torch.int64, device=dev)
    flags = torch.zeros(1, dtype=torch.int32, device=dev)
    kev = []  # (start, end) events around every masking launch of the timed steps (compute stream)

    def step(i, timed_idx=None):
        pipe.run(xs, [1.0] * Lc, gens[i], plan.n_cross, sum_buf, recv, fxp_bits=args.fxp_bits,
                 digests=digests, flags=flags, kernel_events=kev if timed_idx is not None else None)

    for i in range(args.warmup):
        step(i)
    torch.cuda.synchronize()
    if multi:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(args.steps):
        step(args.warmup + i, i)
    torch.cuda.synchronize()
    if multi:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in kev) / args.steps  # masking kernel time per step
    if multi:
        t = torch.tensor([elapsed, kern_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms = float(t[0]), float(t[1])
    if int(flags.item()):
        print("warning: PRG zero-draw flag raised", file=sys.stderr)

    ms_per_step = elapsed * 1e3 / args.steps
    value = C * N / (ms_per_step / 1e3)
    draws = (len(plan.pairs) + len(plan.cross)) * N
    bytes_alg = 4 * Lc * N + 8 * N  # fp32 reads of the local clients + one u64 sum write
    achieved = bytes_alg / (kern_ms / 1e3) / 1e9
    kname = f"k_clients<float, float, {Lc}, {plan.n_cross}>"  # the launch's kernel
    # PMC bytes were collected on the default single-GPU workload only
    pmc = pmc_traffic(f"void sa::{kname}") if (world, C, N) == (1, 8, 100_000_000) else None
    out = {
        "metric": "grad elems/s device-resident: 100M-float quantize+mask+sum, 8 clients",
        "value": value,
        "unit": "grad elems/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": ms_per_step,
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (N(0,0.01^2) fp32 gradients generated on device)",
        "config": {"workload": f"{C} clients x {N} fp32 grad elems, fxp {args.fxp_bits}, ring 2^64, "
                               f"{'1 GPU fused' if world == 1 else f'{Lc} clients/GPU + RCCL reduce'}",
                   "clients": C, "elems_per_client": N, "clients_per_gpu": Lc,
                   "parallelism": f"clients{world}", "pipeline_chunks": len(pipe.bounds)},
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS,
                     "traffic": pmc["bytes"] if pmc else None, "traffic_detail": pmc,
                     "kernel": f"{kname} (sa_fused_clients)", "kernel_ms": kern_ms,
                     "launches_per_step": len(pipe.bounds),
                     "algorithmic_bytes_per_launch": bytes_alg,
                     "valu": {"pcg64_draws_per_launch": draws, "draws_per_s": draws / (kern_ms / 1e3),
                              "peak_draws_per_s": PCG_PEAK_DRAWS,
                              "frac": draws / (kern_ms / 1e3) / PCG_PEAK_DRAWS}},
    }
    if args.extra and world == 1:
        out["extra"] = extra_measurements(args, xs, plan, gens, K, torch, dev)
    if rank == 0:
        out["cpu_baseline"] = cpu
    if rank == 0:
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()
        dist.destroy_process_group()


def extra_measurements(args, xs, plan, gens, K, torch, dev) -> dict:
    """Wire-faithful chain (each client's masked vector materialised, then the
    server sum) and the host-resident rate (H2D of fp32 inputs + D2H of the
    masked vectors, pinned buffers), both on one GPU."""
    from sfl_amd import _lib as L

    C, N = args.clients, args.elems
    names = [f"client{c}" for c in range(C)]
    outs = [torch.empty(N, dtype=torch.int64, device=dev) for _ in range(C)]
    s = torch.empty(N, dtype=torch.int64, device=dev)

    def wire():
        for c in range(C):
            st = [(L.pcg64_from_seed(pair_seed(c, v)), 1 if names[v] > names[c] else -1, v)
                  for v in range(C) if v != c]
            K.mask(xs[c], outs[c], st)
        K.sum_u64(outs, s)

    wire()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    reps = 3
    for _ in range(reps):
        wire()
    torch.cuda.synchronize()
    t_wire = (time.perf_counter() - t0) / reps
    res = {"wire_chain_ms": t_wire * 1e3, "wire_chain_grad_elems_per_s": C * N / t_wire}

    host_x = [x.cpu().pin_memory() for x in xs]
    host_m = [torch.empty(N, dtype=torch.int64).pin_memory() for _ in range(C)]
    dev_x = [torch.empty_like(x) for x in xs]
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for c in range(C):
        dev_x[c].copy_(host_x[c], non_blocking=True)
        st = [(L.pcg64_from_seed(pair_seed(c, v)), 1 if names[v] > names[c] else -1, v)
              for v in range(C) if v != c]
        K.mask(dev_x[c], outs[c], st)
        host_m[c].copy_(outs[c], non_blocking=True)
    torch.cuda.synchronize()
    t_h = time.perf_counter() - t0
    res.update({"host_resident_ms": t_h * 1e3, "host_resident_grad_elems_per_s": C * N / t_h,
                "host_resident_note": "H2D fp32 in + mask + D2H u64 masked vector per client, pinned, one stream"})
    return res


if __name__ == "__main__":
    main()
