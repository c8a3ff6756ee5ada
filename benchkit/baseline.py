"""bench.py's CPU baseline: the oracle's numpy restatement
of the path timed on this host's cores on a bounded sample of the same
workload -- single-threaded, and one process per client.  Measurement
infrastructure: only bench.py's ``cpu_baseline`` leg runs the oracle."""

from __future__ import annotations

import json
import os
import time


def pair_seed(u: int, v: int) -> int:
    a, b = (u, v) if u < v else (v, u)
    return (0x5ECA66 << 32) | (a << 16) | b


def cpu_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    import platform

    return platform.processor() or "unknown"


def cpu_baseline(C: int, fxp_bits: int, seconds: float, parallel: bool = True) -> dict:
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
    par = None
    if parallel:
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
            "cpu_model": cpu_model(), "cores_available": cores,
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


def rank_cpu_seconds(args, world: int) -> float:
    """CPU-baseline budget: the full sample at N=1; a short single-threaded
    one at N>1 so the scaling runs stay short (it delays rank 0 only)."""
    return args.cpu_baseline_seconds if world == 1 else min(3.0, args.cpu_baseline_seconds)


def rank_cpu_baseline(args, world: int, rank: int):
    """rank 0's CPU baseline, always measured before this process touches the
    GPU: handed over by the launcher (launch_ranks) or measured here."""
    if rank != 0 or args.cpu_baseline_seconds <= 0:
        return None
    path = os.environ.get("SFL_BENCH_CPU_BASELINE")
    if path and os.path.exists(path):
        with open(path) as f:
            return json.load(f)
    return cpu_baseline(args.clients, args.fxp_bits, rank_cpu_seconds(args, world), parallel=world == 1)
