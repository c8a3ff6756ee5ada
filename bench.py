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
N>1: one process per GPU, clients sharded in contiguous blocks (8/N per
GPU, config 3 at N=8); each rank runs the fused masking over its clients
(internal pairs + cross streams), pipelined in chunks against ncclReduce of
the uint64 partial sums to rank 0 (the server) over xGMI.  Total work is
fixed as N grows: "scaling": "strong".  `--exchange sharded` replaces the
reduce with the sharded server of SURVEY.md §8(e) (ncclReduceScatter, every
rank decodes its shard; `--gather` also gathers the float64 shards to rank 0).  `python bench.py --gpus N` starts
its N rank processes itself (torch.distributed.run as a child process,
before this process touches the GPU); under an outer torchrun (WORLD_SIZE
set) it runs as one rank.

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
# PCG64 draw-loop ceilings (tools/microbench/draw_issue.hip,
# profiles/r01/draw_issue_microbench.txt), the draw loop alone with the
# product kernel's operand layout and schedule; the first is measured live on
# the bench's own box when the tool is built (draw_loop_ceiling), this
# constant is the fallback:
PCG_PAIR_DRAWS_2WAVE = 1.34e12  # pair draws (both ends accumulated), 2 waves/SIMD = the L=8 kernel's
                                # occupancy ("dual pair28 E2", best of 1.29-1.34e12 run to run)
PCG_ONE_DRAWS_8WAVE = 1.57e12   # one-sided draws at 8 waves/SIMD ("dual one7 E2")


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


PMC_DIRS = [os.path.join(ROOT, "profiles", r) for r in ("r02", "r01")]  # newest first
PMC_ELEMS = 100_000_000  # element positions per launch of the committed PMC passes


def pmc_traffic(kernel: str, elems_per_launch: int) -> dict | None:
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (tools/gpu_profile.sh: separate FETCH_SIZE / WRITE_SIZE runs of
    tools/kernel_bench.py, every per-rank shape at 100M element positions per
    launch), scaled to this run's launch size (the kernel streams: its bytes
    are linear in the element count).  Units are KiB; gfx950 reports
    FETCH_SIZE at half the bytes of 16-B/lane streaming reads, so it is
    doubled (MI355X_MICROARCH.md, HBM); both corrections were checked on the
    k_sum_u64 calibration launch in the same runs (known bytes)."""
    import csv
    import re

    def shape(name):  # (L, X) of a k_clients kernel name; its variant K moves the same bytes
        m = re.search(r"k_clients<float, float, (\d+), (\d+)(?:, (\d+))?>", name)
        return (int(m.group(1)), int(m.group(2))) if m else None

    want = shape(kernel)
    for d in PMC_DIRS:
        vals = {}
        for counter, fname, scale in (("FETCH_SIZE", "pmc_fetch_size.csv", 2.0),
                                      ("WRITE_SIZE", "pmc_write_size.csv", 1.0)):
            path = os.path.join(d, fname)
            if not os.path.exists(path):
                break
            with open(path) as f:
                v = [float(r["Counter_Value"]) for r in csv.DictReader(f)
                     if want is not None and shape(r["Kernel_Name"]) == want and r["Counter_Name"] == counter]
            if not v:
                break
            vals[counter] = scale * 1024.0 * sum(v) / len(v) * elems_per_launch / PMC_ELEMS
        if len(vals) == 2:
            return {"bytes": vals["FETCH_SIZE"] + vals["WRITE_SIZE"], "read": vals["FETCH_SIZE"],
                    "write": vals["WRITE_SIZE"],
                    "source": os.path.relpath(d, ROOT) + "/pmc_{fetch,write}_size.csv",
                    "scaled_from_elems": PMC_ELEMS}
    return None


# k_clients' variant flags (sfl_amd/csrc/sa_internal.h): the instantiation a
# fused launch takes, as sa_fused_clients dispatches it
K_LEAN1, K_SUM_ONLY = 2, 4
SUM_ONLY_SHAPES = {(2, 0), (3, 0), (4, 0), (5, 0), (6, 0), (7, 0), (8, 0), (4, 4), (2, 6), (2, 2), (1, 1), (1, 3), (1, 7)}


def kernel_variant(L: int, X: int, digests: bool) -> int:
    lean = K_LEAN1 if L == 1 else 0
    if not digests and (L, X) in SUM_ONLY_SHAPES:
        return lean | K_SUM_ONLY
    return lean


def _free_port() -> int:
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(args) -> int:
    """`--gpus N` without an outer torchrun (WORLD_SIZE unset): measure the CPU
    baseline here, then start the N rank processes as ONE child process
    (torch.distributed.run, rendezvous on 127.0.0.1) and return its exit
    code.  This process never touches the GPU (it imports no torch), so
    nothing is exec'd from a process that initialised HIP."""
    import subprocess
    import tempfile

    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    tmp = None
    if args.cpu_baseline_seconds > 0:
        cpu = cpu_baseline(args.clients, args.fxp_bits, rank_cpu_seconds(args, args.gpus),
                           parallel=args.gpus == 1 and not args.dry_run)
        fd, tmp = tempfile.mkstemp(prefix="sfl_bench_cpu_", suffix=".json")
        with os.fdopen(fd, "w") as f:
            json.dump(cpu, f)
        env["SFL_BENCH_CPU_BASELINE"] = tmp
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(args.gpus),
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()), os.path.abspath(__file__),
           *sys.argv[1:]]
    try:
        return subprocess.run(cmd, env=env).returncode
    finally:
        if tmp:
            os.unlink(tmp)


def draw_loop_ceiling() -> dict | None:
    """The PCG64 draw loop alone with the 8-client kernel's operand layout,
    schedule and occupancy (tools/microbench/draw_issue, "dual pair28 E2" at
    2 waves/SIMD: median of 15 launches after 40 warm-up ones), measured on THIS box in a child
    process before this process touches the GPU, so roofline.valu compares
    the kernel with a same-box ceiling (boards differ by a few % in clock
    under the power limit).  None if the tool is missing or fails."""
    import subprocess

    exe = os.path.join(ROOT, "tools", "microbench", "draw_issue")
    if not os.path.exists(exe):
        return None
    try:
        r = subprocess.run([exe, "dual pair28 E2", "2"], capture_output=True, text=True, timeout=120)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
        return json.loads(line)
    except (subprocess.SubprocessError, IndexError, ValueError, OSError):
        return None


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


def dry_run(args, world: int, rank: int, cpu) -> None:
    """Launcher rehearsal without a GPU (tests/test_bench_launcher.py): every
    rank joins a gloo group and reports its pid; rank 0 prints one line."""
    import torch.distributed as dist

    multi = world > 1 or args.dist
    ranks = [{"rank": rank, "pid": os.getpid(), "local_rank": int(os.environ.get("LOCAL_RANK", "0"))}]
    if multi:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        allr = [None] * world
        dist.all_gather_object(allr, ranks[0])
        ranks = allr
        dist.destroy_process_group()
    if rank == 0:
        print(json.dumps({"metric": METRIC, "value": None, "dry_run": True, "n_gpus": world, "ranks": ranks,
                          "config": {"workload": workload(args, world)}, "cpu_baseline": cpu}), flush=True)


METRIC = "grad elems/s device-resident: 100M-float quantize+mask+sum, 8 clients"


def workload(args, world: int) -> str:
    from sfl_amd.parallel_sum import client_shard

    C, N = args.clients, args.elems
    if (world > 1 or args.dist) and args.shard == "elements":
        return (f"{C} clients x {N} fp32 grad elems over {world} GPUs, element-sharded: every rank masks its "
                f"1/{world} of every client's elements in one fused launch k_clients<float,float,{C},0> "
                f"({C * (C - 1) // 2} pair streams jumped to the slice start), decodes its slice of the sum"
                + (", float64 slices gathered to rank 0" if args.gather else ""))
    L = len(client_shard(C, world, 0))
    X = C - L
    pairs = L * (L - 1) // 2
    if world == 1:
        if L > 8 and X == 0 and not args.digests:  # the pair-shared multi-launch schedule
            from sfl_amd.kernels import many_schedule

            groups, blocks = many_schedule(C)
            return (f"{C} clients x {N} fp32 grad elems on 1 GPU, fxp {args.fxp_bits}, ring 2^64: pair-shared "
                    f"schedule, every pair stream expanded once ({pairs} pair streams): {len(groups)} "
                    f"k_clients<float,float,<=8,0> launches (the groups' clients and internal pairs) + "
                    f"{len(blocks)} k_clients<float,float,8,0,1> launches (two quads' cross pairs, "
                    f"sa_fused_bipartite), all adding into the sum")
        if L > 8 or pairs + L * X > 32:  # beyond sa_fused_clients' shapes: client by client
            return (f"{C} clients x {N} fp32 grad elems on 1 GPU, fxp {args.fxp_bits}, ring 2^64: per-client "
                    f"sa_mask passes of <= 16 streams accumulating into the sum ({C - 1} streams per client, "
                    f"no pair sharing)")
        return (f"{C} clients x {N} fp32 grad elems on 1 GPU, fxp {args.fxp_bits}, ring 2^64: one fused launch "
                f"k_clients<float,float,{L},{X}> ({pairs} pair streams)")
    return (f"{C} clients x {N} fp32 grad elems over {world} GPUs, fxp {args.fxp_bits}, ring 2^64; per rank: "
            f"{L} local client(s), {pairs} internal pair + {L * X} cross streams "
            f"(k_clients<float,float,{L},{X}>), pipelined " +
            ("ncclReduceScatter(uint64) of the partial sum, each rank decoding its shard (sharded server)"
             + (" and gathering the float64 shards to rank 0" if args.gather else "")
             if args.exchange == "sharded" else "ncclReduce(uint64) of the partial sum to rank 0"))


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--gpus", type=int, default=1)
    # 2000 timed steps (~4.3 s of kernels at N=1, ~5-30 s at N>1 where the
    # exchange bounds a step): long enough for an outside utilisation sampler
    # to catch the GPU busy; 20 warm-up steps cover the
    # clock ramp after idle (the first ~8 launches run long)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--warmup", type=int, default=20)
    ap.add_argument("--clients", type=int, default=8)
    ap.add_argument("--elems", type=int, default=100_000_000)
    ap.add_argument("--fxp-bits", type=int, default=18)
    ap.add_argument("--cpu-baseline-seconds", type=float, default=10.0, help="0 disables")
    ap.add_argument("--extra", action="store_true", help="also time the wire chain and H2D/D2H-inclusive rate")
    ap.add_argument("--dist", action="store_true",
                    help="run the multi-GPU code path (RCCL communicator, reduce) even at N=1 "
                         "(rehearsal of the N>1 path on one GPU)")
    ap.add_argument("--chunks", type=int, default=None,
                    help="masking/reduce pipeline depth (default 8 for N>1, 1 at N=1)")
    ap.add_argument("--exchange", choices=("reduce", "sharded"), default="reduce",
                    help="N>1 exchange: ncclReduce of the partial sums to rank 0 (default), or the sharded "
                         "server of SURVEY.md 8(e): ncclReduceScatter, every rank decodes its shard")
    ap.add_argument("--gather", action="store_true",
                    help="with --exchange sharded or --shard elements: also gather the decoded float64 shards "
                         "to rank 0")
    ap.add_argument("--shard", choices=("clients", "elements"), default="clients",
                    help="N>1: clients in contiguous blocks per GPU (default, config 3), or every GPU takes "
                         "1/N of every client's elements (SURVEY.md 8(e)'s alternative; no exchange for the sum)")
    ap.add_argument("--digests", action="store_true",
                    help="also fold every client's masked values into an XOR digest (test checksum)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher rehearsal without a GPU: ranks join a gloo group, rank 0 prints one line")
    ap.add_argument("--watchdog-seconds", type=float, default=900.0,
                    help="a rank still running after this long exits with status 3 (a hung collective "
                         "cannot be interrupted from Python; torchrun then stops the other ranks); 0 disables")
    args = ap.parse_args()

    if "WORLD_SIZE" not in os.environ and (args.gpus > 1 or args.dist):
        sys.exit(launch_ranks(args))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if args.watchdog_seconds > 0:
        import threading

        def _expire():
            print(f"bench.py rank {rank}: still running after {args.watchdog_seconds:.0f} s, exiting",
                  file=sys.stderr, flush=True)
            os._exit(3)

        wd = threading.Timer(args.watchdog_seconds, _expire)
        wd.daemon = True
        wd.start()
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # CPU baseline first: its per-client worker processes are forked, which
    # must happen before this process initialises the GPU
    cpu = rank_cpu_baseline(args, world, rank)
    if args.dry_run:
        dry_run(args, world, rank, cpu)
        return
    # same-box draw-loop ceiling (N = 1: the headline's 8-client kernel),
    # also before this process initialises the GPU
    ceiling = draw_loop_ceiling() if world == 1 and not args.dist and args.clients == 8 else None

    import torch
    import torch.distributed as dist

    from sfl_amd import _lib
    from sfl_amd import kernels as K
    from sfl_amd.parallel_sum import PipelinedMaskedSum, RcclComm, element_shard, plan_generators, plan_rank

    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
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
    by_elems = multi and args.shard == "elements"
    # element sharding (SURVEY.md §8(e)'s alternative): every rank holds ALL
    # clients' elements [e0, e0 + n_loc) and masks them in one fused launch,
    # streams jumped to e0; no exchange for the sum (each rank's slice of it
    # is complete), the decoded float64 slices gathered to rank 0 on --gather
    plan = plan_rank(names, 1 if by_elems else world, 0 if by_elems else rank)
    Lc = len(plan.clients)
    e0, n_loc, k_el = element_shard(N, world, rank) if by_elems else (0, N, N)
    xs = []
    for c in plan.clients:
        g = torch.Generator(device=dev).manual_seed(20260116 + c)
        x = torch.randn(N, generator=g, device=dev, dtype=torch.float32) * 1e-2
        xs.append(x[e0:e0 + n_loc].clone() if by_elems else x)  # the same data as at N = 1
        del x
    total_steps = args.warmup + args.steps
    chunks = args.chunks if args.chunks is not None else (8 if world > 1 and not by_elems else 1)
    sharded = multi and args.exchange == "sharded" and not by_elems
    pipe = PipelinedMaskedSum(None if by_elems else comm, dev, n_loc, chunks,
                              exchange="sharded" if sharded else "reduce")
    # every step is a new round: streams start i*N draws in, chunk j at +lo_j
    gens = [[plan_generators(plan, pair_seed, offset=i * N + e0 + lo) for lo, _ in pipe.bounds]
            for i in range(total_steps)]
    # the partial sum is reduced IN PLACE (rank 0, the server, receives the
    # masked sum in sum_buf; at N=1 the reduce is a no-op)
    # (sharded server: padded to whole shards, the padding zeroed once; every
    # rank decodes its shard of each chunk into dec on the comm stream)
    sum_buf = torch.zeros(max(pipe.buffer_len, k_el if by_elems else 0), dtype=torch.int64, device=dev)
    dec = torch.zeros(pipe.buffer_len, dtype=torch.float64, device=dev) if sharded else None
    if by_elems:  # this rank's decoded slice (padded to the equal gather count) and rank 0's whole result
        dec = torch.zeros(k_el, dtype=torch.float64, device=dev)
        dec_all = torch.zeros(world * k_el, dtype=torch.float64, device=dev) if rank == 0 and args.gather else None
    # no per-client digests: an XOR checksum the tests use to pin every
    # client's masked vector, not part of the reference's arithmetic; the
    # kernel forms each client's masked value and adds it to the sum either
    # way.  --digests restores them (+1.6 % kernel time).
    digests = torch.zeros(Lc, dtype=torch.int64, device=dev) if args.digests else None
    flags = torch.zeros(1, dtype=torch.int32, device=dev)
    kev = []  # (start, end) events around every masking launch of the timed steps (compute stream)
    xev = []  # (start, end) events around every reduce of the timed steps (comm stream)

    def step(i, timed_idx=None):
        if by_elems:
            pipe.run(xs, [1.0] * Lc, gens[i], 0, sum_buf[:n_loc], None, fxp_bits=args.fxp_bits,
                     digests=digests, flags=flags, kernel_events=kev if timed_idx is not None else None)
            cs = torch.cuda.current_stream(dev)
            if timed_idx is not None:
                xev.append((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
                xev[-1][0].record(cs)
            K.decode(sum_buf[:k_el], dec, fxp_bits=args.fxp_bits)
            if args.gather:
                comm.gather_f64(dec, dec_all, root=0)
            if timed_idx is not None:
                xev[-1][1].record(cs)
            return
        # join=False: a round's exchange tail overlaps the next round's first
        # launches (each chunk's launch still waits for that chunk's previous
        # reduce); the timed region ends with a device synchronise
        pipe.run(xs, [1.0] * Lc, gens[i], plan.n_cross, sum_buf, None, fxp_bits=args.fxp_bits,
                 digests=digests, flags=flags, kernel_events=kev if timed_idx is not None else None,
                 exchange_events=xev if timed_idx is not None else None, join=False,
                 dec=dec, gather=args.gather)

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
    xchg_ms = sum(a.elapsed_time(b) for a, b in xev) / args.steps  # reduce time per step (comm stream)
    if multi:
        t = torch.tensor([elapsed, kern_ms, xchg_ms], dtype=torch.float64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms, xchg_ms = float(t[0]), float(t[1]), float(t[2])
    if int(flags.item()):
        print("warning: PRG zero-draw flag raised", file=sys.stderr)

    ms_per_step = elapsed * 1e3 / args.steps
    value = C * N / (ms_per_step / 1e3)
    draws = (len(plan.pairs) + len(plan.cross)) * n_loc
    bytes_alg = 4 * Lc * n_loc + 8 * n_loc  # per step: fp32 reads of the local clients + one u64 sum write
    launches = len(pipe.bounds)
    achieved = bytes_alg / (kern_ms / 1e3) / 1e9
    kname = f"k_clients<float, float, {Lc}, {plan.n_cross}, {kernel_variant(Lc, plan.n_cross, args.digests)}>"
    n_streams = len(plan.pairs) + len(plan.cross)
    fused = Lc <= 8 and n_streams <= 32  # sa_fused_clients' limits (kMaxLocal, kMaxStreams)
    if not fused and Lc > 8 and plan.n_cross == 0 and not args.digests:  # kernels.fused_many
        kname = (f"pair-shared schedule for {Lc} local clients: k_clients<float, float, 8, 0, 1> "
                 f"(sa_fused_bipartite) + k_clients<float, float, <=8, 0> launches")
    elif not fused:  # sa_fused_clients masks client by client (sa_mask passes of <= 16 streams)
        kname = f"k_clients<float, float, 1, X<=16> per client and pass (fallback for {Lc} local clients)"
    pmc = pmc_traffic(f"void sa::{kname}", n_loc // launches)
    draws_s = draws / (kern_ms / 1e3)
    peak_draws = ceiling["draws_per_s"] if ceiling else PCG_PAIR_DRAWS_2WAVE
    out = {
        "metric": METRIC,
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
        "config": {"workload": workload(args, world),
                   "clients": C, "elems_per_client": N, "clients_per_gpu": Lc,
                   "parallelism": f"{'elements' if by_elems else 'clients'}{world}", "pipeline_chunks": launches,
                   "client_digests": bool(args.digests)},
        # per launch: algorithmic bytes of one launch / its average duration
        # (HIP events on the launch stream); the step's launches are equal
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS,
                     "traffic": pmc["bytes"] if pmc else None, "traffic_detail": pmc,
                     "kernel": f"{kname} (sa_fused_clients)" if fused else kname, "kernel_ms_per_step": kern_ms,
                     "launches_per_step": launches,
                     "algorithmic_bytes_per_launch": bytes_alg / launches,
                     "kernel_ms_per_launch": kern_ms / launches,
                     "valu": {"pcg64_draws_per_step": draws, "draws_per_s": draws_s,
                              "peak_draws_per_s": peak_draws,
                              "peak_source": ("measured on this box: tools/microbench/draw_issue 'dual pair28 E2' "
                                              "at 2 waves/SIMD, median of 15 launches after 40 warm-up" if ceiling else
                                              "constant from profiles/r01/draw_issue_microbench.txt (another box)"),
                              "peak_note": "draw loop alone, pair draws at 2 waves/SIMD (the L=8 kernel's "
                                           "occupancy); one-sided draws at 8 waves/SIMD reach "
                                           f"{PCG_ONE_DRAWS_8WAVE:.3g}",
                              "frac": draws_s / peak_draws,
                              "frac_vs_one_sided_8wave": draws_s / PCG_ONE_DRAWS_8WAVE}},
    }
    if multi:
        # the exchange step: every rank's uint64 partial sum
        # reduced in place to rank 0, one ncclReduce per pipeline chunk on a
        # comm stream beside the masking launches; time from each chunk's
        # launch end on this rank to its reduce end, summed per step, max over
        # ranks.  nccl-tests' convention: reduce bus bandwidth = algbw.
        xb = 8 * N
        coll = "ncclReduce(uint64, sum) in place to rank 0"
        if by_elems:
            xb = 8 * k_el if args.gather else 0
            coll = ("none for the sum (element sharding: each rank's slice of the masked sum is complete); "
                    "k_decode of the slice" + (", float64 slices gathered to rank 0 (ncclSend/Recv)"
                                               if args.gather else ""))
        elif sharded:
            coll = ("sharded server: ncclReduceScatter(uint64, sum) in place, every rank decodes its shard "
                    "(k_decode on the comm stream)" + (", float64 shards gathered to rank 0 (ncclSend/Recv)"
                                                       if args.gather else ""))
        out["exchange"] = {"collective": coll,
                           "chunks": launches, "bytes_per_rank_per_step": xb,
                           "ms_per_step": xchg_ms,
                           "algbw_GBps": xb / (xchg_ms / 1e3) / 1e9 if xchg_ms > 0 and world > 1 else None,
                           "overlap": ("decode (and gather) run after the slice's launch on the compute stream"
                                       if by_elems else "chunk j's reduce runs while chunk j+1 is masked; "
                                       "ms_per_step ~ max(kernel, exchange) + one chunk of fill/drain")}
        if world == 1:
            out["exchange"]["note"] = "world 1 (--dist rehearsal): the collectives move no data between GPUs"
    if args.extra and world == 1:
        out["extra"] = extra_measurements(args, xs, plan, gens, K, torch, dev)
    if rank == 0:
        out["cpu_baseline"] = cpu
        print(json.dumps(out), flush=True)
    if comm is not None:
        comm.close()
        dist.destroy_process_group()


def extra_measurements(args, xs, plan, gens, K, torch, dev) -> dict:
    """Secondary rates on one GPU, none of them `value`:

    * wire chain: every client's masked vector materialised by its own
      sa_mask launch (7 streams each, no pair sharing), then sa_sum_u64;
    * fused wire images: the fused launch storing every client's masked
      vector as well (pair streams still expanded once);
    * host-resident (PCIe-inclusive): fp32 inputs in pinned host memory,
      results back in pinned host memory, chunked so that H2D, the fused
      launch + decode and D2H overlap on three streams; once with only the
      decoded float64 aggregate coming back, once also with every client's
      masked u64 vector (the wire images a loopback party would send);
    * the round-1 serial variant (per client H2D -> sa_mask -> D2H, one
      stream) for comparison."""
    from sfl_amd import _lib as L
    from sfl_amd.parallel_sum import chunk_bounds

    C, N = args.clients, args.elems
    names = [f"client{c}" for c in range(C)]
    outs = [torch.empty(N, dtype=torch.int64, device=dev) for _ in range(C)]
    s = torch.empty(N, dtype=torch.int64, device=dev)
    res = {}

    def timeit(fn, reps=3):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / reps

    def client_streams(c):
        return [(L.pcg64_from_seed(pair_seed(c, v)), 1 if names[v] > names[c] else -1, v)
                for v in range(C) if v != c]

    def wire():
        for c in range(C):
            K.mask(xs[c], outs[c], client_streams(c))
        K.sum_u64(outs, s)

    t = timeit(wire)
    # SURVEY.md 8(d)'s wire-faithful bytes: per client 4 B read + 8 B written
    # (sa_mask), 8 B read again by the server sum, plus the 8-B sum written
    res.update({"wire_chain_ms": t * 1e3, "wire_chain_grad_elems_per_s": C * N / t,
                "wire_chain_algorithmic_GBps": (20 * C * N + 8 * N) / t / 1e9})
    pg, ps, cross = plan_generators_full(plan)

    def fused_wire():
        K.fused_clients(xs, [1.0] * C, pg, ps, cross, plan.n_cross, s, masked_outs=outs)

    t = timeit(fused_wire)
    res.update({"fused_wire_images_ms": t * 1e3, "fused_wire_images_grad_elems_per_s": C * N / t,
                "fused_wire_images_algorithmic_GBps": (12 * C * N + 8 * N) / t / 1e9})

    # ---- host-resident, overlapped
    host_x = torch.stack([x.cpu() for x in xs]).pin_memory()        # [C, N] fp32
    host_dec = torch.empty(N, dtype=torch.float64).pin_memory()
    host_m = torch.empty((C, N), dtype=torch.int64).pin_memory()
    dev_x = torch.empty((C, N), dtype=torch.float32, device=dev)
    dec = torch.empty(N, dtype=torch.float64, device=dev)
    s_h2d, s_cmp, s_d2h = torch.cuda.Stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    bounds = chunk_bounds(N, 16)
    cg = [plan_generators_full(plan, lo) for lo, _ in bounds]

    def host_round(with_images: bool):
        for j, (lo, hi) in enumerate(bounds):
            e_in, e_k = torch.cuda.Event(), torch.cuda.Event()
            with torch.cuda.stream(s_h2d):
                for c in range(C):  # contiguous rows: one DMA each (a 2-D slice would be staged)
                    dev_x[c, lo:hi].copy_(host_x[c, lo:hi], non_blocking=True)
                e_in.record(s_h2d)
            with torch.cuda.stream(s_cmp):
                s_cmp.wait_event(e_in)
                p, sg, cr = cg[j]
                K.fused_clients([dev_x[c, lo:hi] for c in range(C)], [1.0] * C, p, sg, cr, plan.n_cross, s[lo:hi],
                                masked_outs=[o[lo:hi] for o in outs] if with_images else None)
                K.decode(s[lo:hi], dec[lo:hi])
                e_k.record(s_cmp)
            with torch.cuda.stream(s_d2h):
                s_d2h.wait_event(e_k)
                host_dec[lo:hi].copy_(dec[lo:hi], non_blocking=True)
                if with_images:
                    for c in range(C):
                        host_m[c, lo:hi].copy_(outs[c][lo:hi], non_blocking=True)

    for with_images in (False, True):
        t = timeit(lambda: host_round(with_images), reps=2)
        key = "host_resident_with_wire_images" if with_images else "host_resident"
        h2d, d2h = 4 * C * N, 8 * N + (8 * C * N if with_images else 0)
        res.update({f"{key}_ms": t * 1e3, f"{key}_grad_elems_per_s": C * N / t,
                    f"{key}_pcie_bytes": {"h2d": h2d, "d2h": d2h}})
    res["host_resident_note"] = ("pinned host fp32 inputs -> H2D -> fused quantize+mask+sum -> decode -> D2H of the "
                                 "float64 aggregate (and of every client's masked u64 vector), 16 chunks, H2D / "
                                 "compute / D2H on three streams")

    # ---- round-1 serial variant
    host_m1 = [host_m[c] for c in range(C)]

    def serial():
        for c in range(C):
            dev_x[c].copy_(host_x[c], non_blocking=True)
            K.mask(dev_x[c], outs[c], client_streams(c))
            host_m1[c].copy_(outs[c], non_blocking=True)

    t = timeit(serial, reps=1)
    res.update({"host_serial_ms": t * 1e3, "host_serial_grad_elems_per_s": C * N / t,
                "host_serial_note": "H2D fp32 in + sa_mask + D2H u64 masked vector per client, one stream"})
    return res


def plan_generators_full(plan, offset: int = 0):
    from sfl_amd.parallel_sum import plan_generators

    return plan_generators(plan, pair_seed, offset=offset)


if __name__ == "__main__":
    main()
