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
(internal pairs + cross streams), pipelined in chunks against the exchange
of the uint64 partial sums over xGMI.  `value` is measured on the sharded
server (every rank receives and decodes its shard of the
masked sum), its exchange done by ncclReduceScatter in place -- measured
FIRST, before any other design; the same process group then times every
other design (`exchange_variants`: the shards also gathered to rank 0, the
sharded server over direct shard transfers, ncclReduce of the partial sums
to rank 0, element sharding with and without the gather), each contained:
a design that raises is recorded with its error, one that hangs past
--variant-timeout makes rank 0 print the line so far (the headline stands).
The N > 1 line also carries `rccl`: RCCL's own account from every rank's
init log (benchkit/rccl_log.py) -- the transport of every connection
(P2P/IPC over xGMI, SHM or NET/Socket), the ranks and nodes it saw -- and
ncclCommCount / ncclCommCuDevice of our communicator (sa_comm_info).
Total work is fixed as N grows:
"scaling": "strong".  `python bench.py --gpus N` starts its N rank
processes itself (torch.distributed.run as a child process with a c10d
rendezvous on 127.0.0.1 port 0, before this process touches the GPU; a
failing rank's traceback is printed at the end); under an outer torchrun
(WORLD_SIZE set) it runs as one rank.  A rank still running after
--watchdog-seconds (480) without a headline dumps every thread's stack and
exits 1.

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

from benchkit.baseline import cpu_baseline, pair_seed, rank_cpu_baseline, rank_cpu_seconds  # noqa: E402,F401
from benchkit.containment import (Watchdog, control_group, inject_in_design, injected, publish_error,  # noqa: E402,F401
                                  published_errors, run_contained, run_variants, variant_summary)
from benchkit.launcher import failing_ranks_report, launch_ranks  # noqa: E402,F401
from benchkit import rccl_log  # noqa: E402
from benchkit.roofline import (HBM_PEAK_GBPS, PCG_ONE_DRAWS_8WAVE, PCG_PAIR_DRAWS_2WAVE,  # noqa: E402,F401
                               PMC_DIRS, PMC_ELEMS, VALU_PEAK_WAVE_INSTR_PER_S, committed_kernel_ms,
                               draw_loop_ceilings, exchange_model, kernel_key, pmc_traffic, pmc_valu,
                               traffic_field)
from benchkit.standin import HostStandinComm, one_gpu_rccl_comm, one_gpu_rccl_env  # noqa: E402,F401


# k_clients' variant flags (sfl_amd/csrc/sa_internal.h): the instantiation a
# fused launch takes, as sa_fused_clients dispatches it
K_LEAN1, K_SUM_ONLY = 2, 4
SUM_ONLY_SHAPES = {(2, 0), (3, 0), (4, 0), (5, 0), (6, 0), (7, 0), (8, 0), (4, 4), (2, 6), (2, 2), (1, 1), (1, 3), (1, 7)}


CROSS_COUNTS = (32, 24, 16, 8, 4, 2, 1)  # kCrossCounts (sfl_amd/csrc/sa_internal.h)
K_CROSS_ONLY = 8


def multi_launch_plan(L: int, X: int) -> tuple[int, list[int]] | None:
    """sa_fused_clients' multi-launch schedule for a per-rank shape beyond one
    launch (L <= 8 local clients, sum only): (X1, masks-only launch sizes) --
    the first fused sum-only launch takes the internal pairs and the first X1
    cross streams of every client (the largest X1 < X with a sum-only
    instantiation and at most 32 streams), the rest go in launches of the
    largest kCrossCounts that fits.  None when one launch holds the shape
    (or none can: L > 8)."""
    pi = L * (L - 1) // 2
    if L > 8 or pi + L * X <= 32:
        return None
    x1 = next((x for x in range(X - 1, -1, -1) if pi + L * x <= 32 and (L, x) in SUM_ONLY_SHAPES), None)
    if x1 is None:
        return None
    rest, sizes = L * (X - x1), []
    while rest:
        c = next(c for c in CROSS_COUNTS if c <= rest)
        sizes.append(c)
        rest -= c
    return x1, sizes


def multi_launch_text(L: int, X: int) -> str:
    x1, sizes = multi_launch_plan(L, X)
    return (f"pair-shared multi-launch schedule: k_clients<float,float,{L},{x1}> (the "
            f"{L * (L - 1) // 2} internal pairs once + {L * x1} cross streams) then {len(sizes)} masks-only "
            f"k_clients<float,float,1,X,{K_LEAN1 | K_SUM_ONLY | K_CROSS_ONLY}> launches (X = "
            f"{'+'.join(str(c) for c in sizes)} cross streams) adding into the sum")


def kernel_variant(L: int, X: int, digests: bool) -> int:
    lean = K_LEAN1 if L == 1 else 0
    if not digests and (L, X) in SUM_ONLY_SHAPES:
        return lean | K_SUM_ONLY
    return lean


# ---------------------------------------------------------------- N > 1 designs
#
# Every N > 1 run measures ALL of these in one process group (the headline
# first, with --steps; the rest with --variant-steps), so one driver run of
# `bench.py --gpus N` reports each exchange design:
#   sharded          client sharding, every chunk's uint64 partial sum
#                    ncclReduceScatter'ed in place, each rank decodes its shard
#                    (the sharded server) -- the default
#   sharded+gather   ... and the float64 shards gathered to rank 0
#   direct           the sharded server with the reduce-scatter done as direct
#                    shard transfers (grouped ncclSend/Recv: each shard crosses
#                    one xGMI link) + a local k_sum_u64 of the W shards
#   reduce           client sharding, ncclReduce of the partial sums to rank 0
#   elements         element sharding: every rank masks 1/N of EVERY client's
#                    elements, no exchange for the sum (not config 3: a
#                    client's raw gradient on every GPU), decodes its slice
#   elements+gather  ... and the float64 slices gathered to rank 0
VARIANTS = ("sharded", "sharded+gather", "direct", "reduce", "elements", "elements+gather")


class Variant:
    def __init__(self, name: str):
        if name not in VARIANTS and name not in ("local", "direct+gather"):
            raise ValueError(f"unknown exchange variant {name!r}")
        self.name = name
        self.shard = "elements" if name.startswith("elements") else "clients"
        self.exchange = name.split("+")[0] if self.shard == "clients" and name != "local" else None
        self.gather = name.endswith("+gather")


def headline_variant(args, multi: bool) -> Variant:
    """The design `value` is measured on: one fused launch at N = 1; at N > 1
    (or --dist) the one the flags name, the sharded server by default."""
    if not multi:
        return Variant("local")
    if args.shard == "elements":
        return Variant("elements+gather" if args.gather else "elements")
    ex = args.exchange or "sharded"
    return Variant(f"{ex}+gather" if ex in ("sharded", "direct") and args.gather else ex)


def other_variants(args, head: Variant) -> list[Variant]:
    if args.variants == "none":
        return []
    names = VARIANTS if args.variants == "all" else tuple(v for v in args.variants.split(",") if v)
    return [Variant(v) for v in names if v != head.name]


def dry_run(args, world: int, rank: int, cpu, wd: Watchdog) -> None:
    """Launcher rehearsal without a GPU (tests/test_bench_launcher.py): every
    rank joins a gloo group and reports its pid, then the N > 1 design
    sequence runs as on the GPU -- the headline first, every other design
    contained by run_variants and the watchdog -- with dry_design's gloo
    steps in place of the masking and the exchange; rank 0 prints one line."""
    import torch.distributed as dist

    multi = world > 1 or args.dist
    # what a GPU rank would add to its environment before its communicators
    # (rank_comm_env), and the rehearsal-only RCCL variables it inherited
    comm_env = rank_comm_env(args, rank, multi, "/nonexistent")
    ranks = [{"rank": rank, "pid": os.getpid(), "local_rank": int(os.environ.get("LOCAL_RANK", "0")),
              "master_port": os.environ.get("MASTER_PORT"), "comm_env": sorted(comm_env),
              "inherited_rehearsal_env": sorted(k for k in rccl_log.REHEARSAL_ONLY_ENV if k in os.environ)}]
    if multi:
        dist.init_process_group("gloo", rank=rank, world_size=world)
        allr = [None] * world
        dist.all_gather_object(allr, ranks[0])
        ranks = allr
    ctx = {"args": args, "world": world, "rank": rank}
    head = headline_variant(args, multi)
    wd.enter("headline")
    r = dry_design(ctx, head, args.steps, args.warmup)
    check_local = r.pop("check_local")
    line = {"metric": METRIC, "value": r["value"], "dry_run": True, "check": {"round": 0, "decoded_digest": None},
            "data": "dry run: no GPU; every step one gloo all_reduce of 4 KiB (the control flow, not a rate)",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup, "ms_per_step": r["ms_per_step"],
            "ranks": ranks, "config": {"workload": workload(args, world, head), "design": head.name},
            "cpu_baseline": cpu, "watchdog_seconds": args.watchdog_seconds,
            "variant_timeout_seconds": args.variant_timeout}
    if multi:
        line["designs_agree"] = True
        line["roofline"] = {"exchange": r["exchange"]["model"]}
        line["exchange_variants"] = [dict(variant_summary(r), workload=workload(args, world, head))]
        with wd.lock:
            wd.line = line if rank == 0 else {}
        settle_check(ctx, r, check_local, line, wd)
        others = other_variants(args, head)

        def summarise(x):
            return dict(variant_summary(x), workload=workload(args, world, Variant(x["name"])))

        run_variants(ctx, dry_design, others, summarise, line, wd, settle=combine_check)
    else:
        line["check"]["decoded_digest"] = f"{check_local:016x}"
    wd.enter("done")
    if rank == 0:
        wd.emit(line)
    if multi:
        dist.destroy_process_group()


METRIC = "grad elems/s device-resident: 100M-float quantize+mask+sum, 8 clients"


def workload(args, world: int, v: Variant) -> str:
    from sfl_amd.parallel_sum import client_shard

    C, N = args.clients, args.elems
    if v.shard == "elements":
        return (f"{C} clients x {N} fp32 grad elems over {world} GPUs, element-sharded: every rank masks its "
                f"1/{world} of every client's elements in one fused launch k_clients<float,float,{C},0> "
                f"({C * (C - 1) // 2} pair streams jumped to the slice start), decodes its slice of the sum"
                + (", float64 slices gathered to rank 0" if v.gather else ""))
    L = len(client_shard(C, world, 0))
    X = C - L
    pairs = L * (L - 1) // 2
    if world == 1 and v.name == "local":
        if L > 8 and X == 0 and not args.digests:  # the pair-shared multi-launch schedule
            from sfl_amd.kernels import many_schedule

            groups, blocks = many_schedule(C)
            return (f"{C} clients x {N} fp32 grad elems on 1 GPU, fxp {args.fxp_bits}, ring 2^64: pair-shared "
                    f"schedule, every pair stream expanded once ({pairs} pair streams): {len(groups)} "
                    f"k_clients<float,float,<=8,0> launches (the groups' clients and internal pairs) + "
                    f"{len(blocks)} k_clients<float,float,8,0,1> launches (two quads' cross pairs, "
                    f"sa_fused_bipartite), all adding into the sum")
        if L <= 8 and not args.digests and multi_launch_plan(L, X):
            return (f"{C} clients x {N} fp32 grad elems on 1 GPU, fxp {args.fxp_bits}, ring 2^64: "
                    + multi_launch_text(L, X))
        if L > 8 or pairs + L * X > 32:  # beyond sa_fused_clients' shapes: client by client
            return (f"{C} clients x {N} fp32 grad elems on 1 GPU, fxp {args.fxp_bits}, ring 2^64: per-client "
                    f"sa_mask passes of <= 16 streams accumulating into the sum ({C - 1} streams per client, "
                    f"no pair sharing)")
        return (f"{C} clients x {N} fp32 grad elems on 1 GPU, fxp {args.fxp_bits}, ring 2^64: one fused launch "
                f"k_clients<float,float,{L},{X}> ({pairs} pair streams)")
    ml = multi_launch_plan(L, X) if not args.digests else None
    return (f"{C} clients x {N} fp32 grad elems over {world} GPUs, fxp {args.fxp_bits}, ring 2^64; per rank: "
            f"{L} local client(s), {pairs} internal pair + {L * X} cross streams "
            f"({multi_launch_text(L, X) if ml else f'k_clients<float,float,{L},{X}>'}), pipelined " +
            {"sharded": "ncclReduceScatter(uint64) of the partial sum, each rank decoding its shard (sharded server)",
             "direct": "direct shard transfers (ncclSend/Recv, uint64) of the partial sum, each rank summing "
                       "and decoding its shard (sharded server)",
             }.get(v.exchange, "ncclReduce(uint64) of the partial sum to rank 0")
            + (" and gathering the float64 shards to rank 0" if v.gather else ""))


def collective_text(v: Variant) -> str:
    if v.shard == "elements":
        return ("none for the sum (element sharding: each rank's slice of the masked sum is complete); "
                "k_decode of the slice" + (", float64 slices gathered to rank 0 (ncclSend/Recv)"
                                           if v.gather else ""))
    if v.exchange == "sharded":
        return ("sharded server: ncclReduceScatter(uint64, sum) in place, every rank decodes its shard "
                "(k_decode on the comm stream)" + (", float64 shards gathered to rank 0 (ncclSend/Recv)"
                                                   if v.gather else ""))
    if v.exchange == "direct":
        return ("sharded server, direct: every shard sent to its server rank over one link (grouped "
                "ncclSend/Recv, uint64), the rank sums the world shards (k_sum_u64) and decodes them "
                "(k_decode), both on the comm stream" + (", float64 shards gathered to rank 0 (ncclSend/Recv)"
                                                        if v.gather else ""))
    return "ncclReduce(uint64, sum) in place to rank 0"


def dry_exchange_model(design: str, world: int, args) -> dict | None:
    """--dry-run: the exchange model with the committed per-rank kernel time
    (no GPU here): what the driver's node should measure for this N."""
    kms, src = committed_kernel_ms(args.clients, world, args.elems)
    m = exchange_model(design, world, args.elems, kms, None, 8, "dry-run")
    if m is not None:
        m["kernel_ms_source"] = src or "none committed for this shape"
    return m


def dry_design(ctx, v: Variant, steps: int, warmup: int, keep: bool = False) -> dict:
    """--dry-run's stand-in for run_design (no GPU): every step is one gloo
    all_reduce of a small CPU tensor among the ranks, timed like a design
    (barrier on both sides, max over ranks), with run_design's result keys
    and the fault injection; its numbers are the control flow's, not a rate."""
    import torch
    import torch.distributed as dist

    args, world, rank = ctx["args"], ctx["world"], ctx["rank"]
    inject_in_design(v.name, rank)
    multi = world > 1
    t = torch.ones(1024)
    for _ in range(warmup):
        if multi:
            dist.all_reduce(t)
    if multi:
        dist.barrier()
    t0 = time.perf_counter()
    for _ in range(steps):
        if multi:
            dist.all_reduce(t)
    if multi:
        dist.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    if multi:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
    ms = float(el[0]) * 1e3 / max(1, steps)
    check = int(injected("corrupt", v.name, rank))  # this rank's part (combine_check adds them)
    return {"name": v.name, "ms_per_step": ms, "value": args.clients * args.elems / max(ms / 1e3, 1e-9),
            "steps": steps, "warmup": warmup, "kernel_ms_per_step": 0.0, "chunks": 1, "kernel": "none (dry run)",
            "exchange": {"ms_per_step": ms, "bytes_per_rank_per_step": 4096, "algbw_GBps": None, "busbw_GBps": None,
                         "collective": "dry run: one gloo all_reduce of 4 KiB per step",
                         "model": dry_exchange_model(v.name, world, args)},
            "check_local": check}


CHECK_NOTE = ("sum over i of mix64(bits(decoded[i])) * (2i + 1) * 0x9E3779B97F4A7C15 mod 2^64 (mix64 = "
              "splitmix64's finalizer, so no bit of the digest is structurally zero) over the decoded float64 "
              "aggregate of round 0 (all C clients, every element), recomputed after the timed region by one more "
              "untimed step of the same design: every design and every N must print the same value (the same "
              "inputs, seeds and stream positions)")


CHECK_MULT = 0x9E3779B97F4A7C15  # odd: the position weight of element i is (2i + 1) * CHECK_MULT mod 2^64
MIX1, MIX2 = 0xBF58476D1CE4E5B9, 0x94D049BB133111EB  # splitmix64's finalizer


def _s64(c: int) -> int:
    """The same 64 bits as a signed int64 (torch has no uint64 arithmetic)."""
    return c - (1 << 64) if c >> 63 else c


def mix64(z):
    """splitmix64's finalizer on an int64 tensor, bit for bit the uint64
    function (logical shifts by masking; int64 products wrap like uint64).
    A decoded value k / 2^18 with |k| < 2^16 has >= 36 trailing zero bits in
    its float64 pattern; after mix64 every bit depends on every input bit."""
    z = (z ^ ((z >> 30) & ((1 << 34) - 1))) * _s64(MIX1)
    z = (z ^ ((z >> 27) & ((1 << 37) - 1))) * _s64(MIX2)
    return z ^ ((z >> 31) & ((1 << 33) - 1))


def position_digest(t, base: int) -> int:
    """sum_i mix64(bits(t[i])) * (2 (base + i) + 1) * CHECK_MULT mod 2^64
    over a float64 device vector whose element i is element base + i of the
    aggregate: position-weighted, so a shard decoded into the wrong place
    changes it (an XOR or plain sum would not see a permutation), and mixed,
    so all 64 bits of the digest carry information (raw bits of decoded
    fixed-point values end in >= 36 zeros, which made the position weight act
    only mod 2^28).  In slices of 2^26 elements to bound the temporaries."""
    import torch

    mult = _s64(CHECK_MULT)
    out, n, step = 0, t.numel(), 1 << 26
    bits = t.view(torch.int64)
    for lo in range(0, n, step):
        hi = min(n, lo + step)
        h = (torch.arange(base + lo, base + hi, device=t.device, dtype=torch.int64) * 2 + 1) * mult
        out = (out + int((mix64(bits[lo:hi]) * h).sum().item())) & ((1 << 64) - 1)
    return out


def result_check(ctx, v: Variant, step, sum_buf, dec, dec_all, sharded: bool, by_elems: bool, e0: int) -> int:
    """This rank's part of the design's round-0 result check (CHECK_NOTE):
    the position digest of the decoded elements this rank holds (zeros
    elsewhere contribute nothing).  No collective here: combine_check adds
    the ranks' parts mod 2^64 once the line it belongs to is safe (the
    headline's line registered with the watchdog)."""
    import torch

    from sfl_amd import kernels as K

    args, rank, dev, comm = ctx["args"], ctx["rank"], ctx["dev"], ctx["comm"]
    step(0, False)
    torch.cuda.synchronize()
    src, base = None, 0
    if by_elems:  # every rank its decoded slice (global start e0); with the gather rank 0 holds them all
        src, base = (dec_all, 0) if v.gather else (dec, e0)
        if v.gather and rank != 0:
            src = None
        if comm is None:  # world 1 without --dist: the slice is the whole vector, not decoded by the step
            src = torch.empty(args.elems, dtype=torch.float64, device=dev)
            K.decode(sum_buf[:args.elems], src, fxp_bits=args.fxp_bits)
    elif sharded:  # every rank decoded its shards in place (zeros elsewhere); with the gather rank 0 all
        src = dec if (not v.gather or rank == 0) else None
    elif rank == 0:  # reduce (and N = 1): rank 0 holds the masked sum
        src = torch.empty(args.elems, dtype=torch.float64, device=dev)
        K.decode(sum_buf[:args.elems], src, fxp_bits=args.fxp_bits)
    x = position_digest(src, base) if src is not None else 0
    if injected("corrupt", v.name, rank):  # SFL_BENCH_INJECT: a wrong result on this rank
        x = (x + 1) & ((1 << 64) - 1)
    return x


def combine_check(ctx, res: dict) -> str:
    """Add the ranks' parts of a design's round-0 result check mod 2^64 (gloo
    control group): a mis-indexed shard transfer or a wrong slot shows as a
    value differing between designs (run_variants flags it) or between N = 1
    and N > 1."""
    import torch.distributed as dist

    x = res.pop("check_local")
    if ctx["world"] > 1 and dist.is_initialized():
        parts = [None] * ctx["world"]
        dist.all_gather_object(parts, x, group=control_group(ctx))
        x = 0
        for p in parts:
            x = None if p is None or x is None else (x + p) & ((1 << 64) - 1)
    res["check_digest"] = None if x is None else f"{x:016x}"
    return res["check_digest"]


def settle_check(ctx, r: dict, check_local: int, out: dict, wd: Watchdog) -> None:
    """The headline's round-0 check, combined over the ranks AFTER its line
    is registered with the watchdog (phase "check": a hang here prints the
    line without the check, an exception leaves the error in its place)."""
    import traceback

    wd.enter("check")
    try:
        r["check_local"] = check_local
        x = combine_check(ctx, r)
    except Exception as e:  # noqa: BLE001 -- the line stands without the check
        traceback.print_exc()
        x = None
        out["check"]["error"] = repr(e)
    with wd.lock:
        out["check"]["decoded_digest"] = x
        out["exchange_variants"][0]["check_digest"] = x


def run_design(ctx, v: Variant, steps: int, warmup: int, keep: bool = False) -> dict:
    """Time `steps` steps (after `warmup`) of design `v` on this rank: the
    masking launches on the compute stream, the design's exchange on the
    comm stream, bracketed by a barrier + device synchronise on both sides;
    elapsed, kernel and exchange times are the max over ranks."""
    import torch
    import torch.distributed as dist

    from sfl_amd import kernels as K
    from sfl_amd.parallel_sum import PipelinedMaskedSum, element_shard, plan_generators, plan_rank

    args, world, rank, dev, comm = ctx["args"], ctx["world"], ctx["rank"], ctx["dev"], ctx["comm"]
    inject_in_design(v.name, rank)
    multi = comm is not None
    C, N = args.clients, args.elems
    by_elems = v.shard == "elements"
    plan = plan_rank(ctx["names"], 1 if by_elems else world, 0 if by_elems else rank)
    Lc = len(plan.clients)
    e0, n_loc, k_el = element_shard(N, world, rank) if by_elems else (0, N, N)
    xs = []
    for c in plan.clients:
        g = torch.Generator(device=dev).manual_seed(20260116 + c)
        x = torch.randn(N, generator=g, device=dev, dtype=torch.float32) * 1e-2
        xs.append(x[e0:e0 + n_loc].clone() if by_elems else x)  # the same data as at N = 1
        del x
    total = warmup + steps
    chunks = args.chunks if args.chunks is not None else (8 if world > 1 and not by_elems else 1)
    sharded = v.exchange in ("sharded", "direct")
    pipe = PipelinedMaskedSum(None if by_elems else comm, dev, n_loc, chunks,
                              exchange=v.exchange if sharded else "reduce")
    # every step is a new round: streams start i*N draws in, chunk j at +lo_j
    gens = [[plan_generators(plan, pair_seed, offset=i * N + e0 + lo) for lo, _ in pipe.bounds]
            for i in range(total)]
    # the partial sum is reduced IN PLACE (rank 0, the server, receives the
    # masked sum in sum_buf; at N=1 there is no exchange); the sharded
    # server's buffers are padded to whole shards, the padding zeroed once,
    # every rank decoding its shard of each chunk into dec on the comm stream
    sum_buf = torch.zeros(max(pipe.buffer_len, k_el if by_elems else 0), dtype=torch.int64, device=dev)
    dec = torch.zeros(pipe.buffer_len, dtype=torch.float64, device=dev) if sharded else None
    dec_all = None
    if by_elems:  # this rank's decoded slice (padded to the equal gather count) and rank 0's whole result
        dec = torch.zeros(k_el, dtype=torch.float64, device=dev)
        dec_all = torch.zeros(world * k_el, dtype=torch.float64, device=dev) if rank == 0 and v.gather else None
    # no per-client digests: an XOR checksum the tests use to pin every
    # client's masked vector, not part of the reference's arithmetic; the
    # kernel forms each client's masked value and adds it to the sum either
    # way.  --digests restores them (+1.6 % kernel time).
    digests = torch.zeros(Lc, dtype=torch.int64, device=dev) if args.digests else None
    flags = torch.zeros(1, dtype=torch.int32, device=dev)
    kev, xev = [], []  # event pairs around every masking launch / exchange of the timed steps
    # one launch per step and nothing else on the stream (N = 1, one chunk):
    # the launches run back to back, so ONE event pair around the timed
    # region gives their average duration; a timing-event pair around every
    # launch would itself open a ~5-10 us gap between launches (rocprof
    # trace: 0 us between warm-up launches, 10 us between timed ones)
    region = not multi and len(pipe.bounds) == 1

    def step(i, timed):
        if by_elems:
            pipe.run(xs, [1.0] * Lc, gens[i], 0, sum_buf[:n_loc], None, fxp_bits=args.fxp_bits,
                     digests=digests, flags=flags, kernel_events=kev if timed else None)
            cs = torch.cuda.current_stream(dev)
            if timed and multi:
                xev.append((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
                xev[-1][0].record(cs)
            if multi:
                K.decode(sum_buf[:k_el], dec, fxp_bits=args.fxp_bits)
                if v.gather:
                    comm.gather_f64(dec, dec_all, root=0)
            if timed and multi:
                xev[-1][1].record(cs)
            return
        # join=False: a round's exchange tail overlaps the next round's first
        # launches (each chunk's launch still waits for that chunk's previous
        # exchange); the timed region ends with a device synchronise
        pipe.run(xs, [1.0] * Lc, gens[i], plan.n_cross, sum_buf, None, fxp_bits=args.fxp_bits,
                 digests=digests, flags=flags, kernel_events=kev if timed and not region else None,
                 exchange_events=xev if timed else None, join=False, dec=dec, gather=v.gather)

    for i in range(warmup):
        step(i, False)
    torch.cuda.synchronize()
    if multi:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    if region:
        kev.append((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
        kev[0][0].record(torch.cuda.current_stream(dev))
    for i in range(steps):
        step(warmup + i, True)
    if region:
        kev[0][1].record(torch.cuda.current_stream(dev))
    torch.cuda.synchronize()
    if multi:
        dist.barrier()
    torch.cuda.synchronize()
    elapsed = time.perf_counter() - t0
    kern_ms = sum(a.elapsed_time(b) for a, b in kev) / steps  # masking kernel time per step
    xchg_ms = sum(a.elapsed_time(b) for a, b in xev) / steps  # exchange time per step (comm stream)
    if multi:
        t = torch.tensor([elapsed, kern_ms, xchg_ms], dtype=torch.float64,
                         device="cpu" if ctx.get("pg_gloo") else dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, kern_ms, xchg_ms = float(t[0]), float(t[1]), float(t[2])
    try:  # the check is extra: a failure here must not cost the design's timing
        check = result_check(ctx, v, step, sum_buf, dec, dec_all, sharded, by_elems, e0)
    except Exception:  # noqa: BLE001
        import traceback

        traceback.print_exc()
        check = None
    flagged = bool(int(flags.item()))
    ms = elapsed * 1e3 / steps
    n_streams = len(plan.pairs) + len(plan.cross)
    kname = f"k_clients<float, float, {Lc}, {plan.n_cross}, {kernel_variant(Lc, plan.n_cross, args.digests)}>"
    fused = Lc <= 8 and n_streams <= 32  # sa_fused_clients' limits (kMaxLocal, kMaxStreams)
    if not fused and Lc > 8 and plan.n_cross == 0 and not args.digests:  # kernels.fused_many
        kname = (f"pair-shared schedule for {Lc} local clients: k_clients<float, float, 8, 0, 1> "
                 f"(sa_fused_bipartite) + k_clients<float, float, <=8, 0> launches")
    elif not fused and not args.digests and multi_launch_plan(Lc, plan.n_cross):
        kname = multi_launch_text(Lc, plan.n_cross)
    elif not fused:  # sa_fused_clients masks client by client (sa_mask passes of <= 16 streams)
        kname = f"k_clients<float, float, 1, X<=16> per client and pass (fallback for {Lc} local clients)"
    res = {"name": v.name, "ms_per_step": ms, "value": C * N / (ms / 1e3), "steps": steps, "warmup": warmup,
           "kernel_ms_per_step": kern_ms, "chunks": len(pipe.bounds), "kernel": kname, "fused": fused,
           "local_clients": Lc, "n_loc": n_loc, "pair_draws": len(plan.pairs) * n_loc,
           "one_sided_draws": len(plan.cross) * n_loc, "zero_draw_flag": flagged, "check_local": check,
           "kernel_timing": ("one HIP event pair on the launch stream around the timed region's back-to-back "
                             "launches" if region else "a HIP event pair around every launch")}
    if multi:
        # bytes each rank hands the exchange per step; algbw as nccl-tests
        # defines it (buffer bytes / time), busbw the per-rank wire bytes
        if by_elems:
            xb = 8 * k_el * world if v.gather else 0
            busbw_f = (world - 1) / world
        elif sharded:
            xb = 8 * pipe.buffer_len
            busbw_f = (world - 1) / world
        else:
            xb = 8 * N
            busbw_f = 1.0
        algbw = xb / (xchg_ms / 1e3) / 1e9 if xchg_ms > 0 and world > 1 and xb else None
        res["exchange"] = {
            "collective": collective_text(v), "chunks": len(pipe.bounds), "bytes_per_rank_per_step": xb,
            "ms_per_step": xchg_ms, "algbw_GBps": algbw, "busbw_GBps": algbw * busbw_f if algbw else None,
            "timing": ("HIP events on the comm stream from each chunk's launch end on this rank to its "
                       "exchange end (waiting for slower peers counts), summed per step, max over ranks"
                       if not by_elems else "HIP events around the slice's decode (and gather) on the "
                       "compute stream, max over ranks"),
            "overlap": ("decode (and gather) run after the slice's launch on the compute stream" if by_elems
                        else "chunk j's exchange runs while chunk j+1 is masked; ms_per_step ~ "
                        "max(kernel, exchange) + one chunk of fill/drain")}
        if world == 1:
            res["exchange"]["note"] = "world 1 (--dist rehearsal): the collectives move no data between GPUs"
        res["exchange"]["model"] = exchange_model(v.name, world, N, kern_ms, xchg_ms, len(pipe.bounds),
                                                  "rehearsal" if ctx.get("rehearse") else "measured")
    if keep:
        ctx["kept"] = {"xs": xs, "plan": plan, "gens": gens}
    else:
        del xs, gens, sum_buf, dec, dec_all, pipe
        torch.cuda.empty_cache()
    return res


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
                    help="run the multi-GPU code path (RCCL communicator, exchange) even at N=1 "
                         "(rehearsal of the N>1 path on one GPU)")
    ap.add_argument("--chunks", type=int, default=None,
                    help="masking/exchange pipeline depth (default 8 for N>1, 1 at N=1)")
    ap.add_argument("--exchange", choices=("reduce", "sharded", "direct"), default=None,
                    help="N>1 headline exchange: the sharded server of SURVEY.md 8(e) (default: "
                         "ncclReduceScatter, every rank decodes its shard), the same server with direct shard "
                         "transfers (grouped ncclSend/Recv) and a local k_sum_u64, or ncclReduce of the partial "
                         "sums to rank 0")
    ap.add_argument("--gather", action="store_true",
                    help="with --exchange sharded or --shard elements: also gather the decoded float64 shards "
                         "to rank 0")
    ap.add_argument("--shard", choices=("clients", "elements"), default="clients",
                    help="N>1: clients in contiguous blocks per GPU (default, config 3), or every GPU takes "
                         "1/N of every client's elements (SURVEY.md 8(e)'s alternative; no exchange for the sum)")
    ap.add_argument("--variants", default="all",
                    help="N>1: the other exchange designs timed after the headline in the same process group "
                         f"('all' = {','.join(VARIANTS)}; a comma list; 'none')")
    ap.add_argument("--variant-steps", type=int, default=None,
                    help="timed steps per extra design (default: min(200, --steps))")
    ap.add_argument("--variant-timeout", type=float, default=120.0,
                    help="N>1: a design after the headline still running after this many seconds is declared "
                         "hung; rank 0 prints the line so far with that design marked, every rank exits 0")
    ap.add_argument("--masking-reserve", type=int, default=0,
                    help="CUs of the masking grid left free for the overlapped exchange kernels "
                         "(sa_set_masking_reserve; tools/overlap_probe.py measured <= 3 %% either way)")
    ap.add_argument("--host-resident-steps", type=int, default=20,
                    help="N>1 with the sharded headline: also time this many steps with inputs and results in "
                         "pinned host memory (H2D / D2H inclusive, line field host_resident; 0: skip)")
    ap.add_argument("--digests", action="store_true",
                    help="also fold every client's masked values into an XOR digest (test checksum)")
    ap.add_argument("--dry-run", action="store_true",
                    help="launcher rehearsal without a GPU: ranks join a gloo group, rank 0 prints one line")
    ap.add_argument("--rehearse-one-gpu", action="store_true",
                    help="N>1 rehearsal on a one-GPU box: every rank on cuda:0, a gloo process group and the "
                         "collectives through a shared host mapping (RCCL refuses two ranks on one GPU); runs "
                         "every design's code path, its timings are not the product's")
    ap.add_argument("--rehearse-comm", choices=("rccl", "standin"), default="rccl",
                    help="--rehearse-one-gpu's data path: the product's RcclComm, the ranks made distinct RCCL "
                         "'nodes' on the one GPU (NCCL_HOSTID per rank; RCCL's socket transport on lo), or the "
                         "host stand-in (benchkit/standin.py)")
    ap.add_argument("--watchdog-seconds", type=float, default=480.0,
                    help="a rank still running after this long exits: with the headline done, rank 0 first "
                         "prints the line so far (Watchdog); before it, faulthandler dumps every thread's stack "
                         "and exits 1 (torchrun then stops the other ranks); below the driver's 600 s lease; "
                         "0 disables")
    args = ap.parse_args()
    if args.variant_steps is None:
        args.variant_steps = max(1, min(200, args.steps))
    for v in (args.variants.split(",") if args.variants not in ("all", "none") else []):
        if v and v not in VARIANTS:
            ap.error(f"--variants: unknown design {v!r} (choose from {', '.join(VARIANTS)})")

    if "WORLD_SIZE" not in os.environ and (args.gpus > 1 or args.dist):
        sys.exit(launch_ranks(args, __file__))
    # a rank: an uncaught exception is written to torchrun's error file, so
    # the launcher's failure summary names this rank and shows its traceback
    from torch.distributed.elastic.multiprocessing.errors import record

    record(rank_main)(args)


def rank_comm_env(args, rank: int, multi: bool, log_dir: str) -> dict:
    """What a rank adds to its environment before its first communicator:
    RCCL's per-rank init log (benchkit/rccl_log.py) on every RCCL path, and
    ONLY under --rehearse-one-gpu (RCCL between ranks that share one GPU) the
    NCCL_HOSTID / NCCL_SOCKET_IFNAME / NCCL_IB_DISABLE that make each rank
    its own RCCL node over sockets -- never on the product path, where they
    would push the exchange off xGMI (tests/test_bench_launcher.py)."""
    if not multi or (args.rehearse_one_gpu and args.rehearse_comm == "standin"):
        return {}
    env = dict(rccl_log.debug_env(rank, log_dir))
    if args.rehearse_one_gpu:
        env.update(one_gpu_rccl_env(rank))
    return env


def rank_main(args):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local_rank = int(os.environ.get("LOCAL_RANK", "0"))
    import faulthandler

    faulthandler.enable(all_threads=True)  # a fatal signal in a rank leaves its stacks in its stderr log
    wd = Watchdog(args.watchdog_seconds, args.variant_timeout, rank)
    if injected("raise", None, rank):
        raise RuntimeError(f"SFL_BENCH_INJECT: rank {rank} fails at start-up")
    if world != args.gpus:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")
    # CPU baseline first: its per-client worker processes are forked, which
    # must happen before this process initialises the GPU
    cpu = rank_cpu_baseline(args, world, rank)
    if args.dry_run:
        dry_run(args, world, rank, cpu, wd)
        return
    multi = world > 1 or args.dist
    # same-box draw-loop ceilings, also before this process initialises the GPU
    rehearse = args.rehearse_one_gpu
    ceil = {} if rehearse else draw_loop_ceilings(local_rank if world > 1 else None)

    import torch
    import torch.distributed as dist

    from sfl_amd import _lib
    from sfl_amd.parallel_sum import RcclComm

    gpu = 0 if rehearse else local_rank
    torch.cuda.set_device(gpu)
    dev = torch.device("cuda", gpu)
    _lib.check(_lib.lib().sa_set_masking_reserve(args.masking_reserve), "sa_set_masking_reserve")
    comm = None
    rccl_dir = None
    if multi and not (rehearse and args.rehearse_comm == "standin"):
        # RCCL's init log, one file per rank (before the first communicator:
        # RCCL reads its debug settings once per process) -> the line's
        # "rccl" record, which transport carried the exchange
        import tempfile

        keep = os.environ.get("SFL_BENCH_RCCL_LOG_DIR")  # keep the logs there (else a temp dir, removed)
        if keep:
            rccl_dir = os.path.join(keep, f"rank{rank}")
            os.makedirs(rccl_dir, exist_ok=True)
        else:
            rccl_dir = tempfile.mkdtemp(prefix=f"sfl_rccl_rank{rank}_")
        env = rank_comm_env(args, rank, multi, rccl_dir)
        if "NCCL_DEBUG_FILE" not in env:
            os.rmdir(rccl_dir)
            rccl_dir = None
        leaked = [k for k in rccl_log.REHEARSAL_ONLY_ENV if k in os.environ and k not in env]
        if leaked:  # the record names them too (rccl.rehearsal_env)
            print(f"warning: rank {rank}: {', '.join(leaked)} set in the environment: RCCL may not use "
                  "xGMI", file=sys.stderr)
        os.environ.update(env)
    if multi and rehearse and args.rehearse_comm == "standin":
        dist.init_process_group("gloo", rank=rank, world_size=world)
        comm = HostStandinComm(rank, world)
    elif multi and rehearse:
        # the product's process group and communicator, every rank its own
        # RCCL node on this one GPU (NCCL_HOSTID, set by rank_comm_env):
        # torch's NCCL group carries the barriers and the timing reductions,
        # as on the node
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        comm = one_gpu_rccl_comm(rank, world)
    elif multi:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)
        comm = RcclComm(rank, world, local_rank)

    C, N = args.clients, args.elems
    ctx = {"args": args, "world": world, "rank": rank, "dev": dev, "comm": comm, "rehearse": rehearse,
           "pg_gloo": multi and dist.get_backend() == "gloo", "names": [f"client{c}" for c in range(C)]}
    head = headline_variant(args, multi)
    wd.enter("headline")
    r = run_design(ctx, head, args.steps, args.warmup, keep=args.extra and world == 1)
    if r["zero_draw_flag"]:
        print("warning: PRG zero-draw flag raised", file=sys.stderr)
    kern_ms, launches = r["kernel_ms_per_step"], r["chunks"]
    n_loc, Lc = r["n_loc"], r["local_clients"]
    bytes_alg = 4 * Lc * n_loc + 8 * n_loc  # per step: fp32 reads of the local clients + one u64 sum write
    achieved = bytes_alg / (kern_ms / 1e3) / 1e9
    pmc = pmc_traffic(f"void sa::{r['kernel']}", n_loc // launches)
    traffic, traffic_detail = traffic_field(pmc, bytes_alg / launches)
    census = pmc_valu(f"void sa::{r['kernel']}", n_loc // launches)
    int_ops = None
    if census is not None:  # VALU issue rate of the timed launches against the chip's issue peak
        rate = census["valu_wave_instr"] * launches / (kern_ms / 1e3)
        int_ops = {"valu_wave_instr_per_launch": census["valu_wave_instr"], "valu_wave_instr_per_s": rate,
                   "valu_lane_ops_per_s": 64 * rate, "peak_valu_wave_instr_per_s": VALU_PEAK_WAVE_INSTR_PER_S,
                   "frac": rate / VALU_PEAK_WAVE_INSTR_PER_S, "source": census["source"],
                   "note": "instructions per launch from the committed SQ census, time from this run's launches; "
                           "the peak is one wave64 VALU instruction per 4 cycles per SIMD at 2.4 GHz (the board "
                           "holds ~2.33 GHz under its power limit, and VOP3 forms issue at 4.2-4.7 cycles)"}
    # VALU: the step's draws against the same-box draw loop at the same draw
    # kinds: ideal time = pair draws / pair ceiling + one-sided / one-sided ceiling
    pair_peak = ceil["pair"]["draws_per_s"] if "pair" in ceil else PCG_PAIR_DRAWS_2WAVE
    one_peak = ceil["one"]["draws_per_s"] if "one" in ceil else PCG_ONE_DRAWS_8WAVE
    draws = r["pair_draws"] + r["one_sided_draws"]
    ideal_s = r["pair_draws"] / pair_peak + r["one_sided_draws"] / one_peak
    out = {
        "metric": METRIC,
        "value": r["value"],
        "unit": "grad elems/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": r["ms_per_step"],
        "higher_is_better": True,
        "scaling": "strong",
        "vs_baseline": None,
        "dtype": "u64",
        "data": "synthetic (N(0,0.01^2) fp32 gradients generated on device)",
        "config": {"workload": workload(args, world, head),
                   "clients": C, "elems_per_client": N, "clients_per_gpu": Lc, "design": head.name,
                   "parallelism": f"{'elements' if head.shard == 'elements' else 'clients'}{world}",
                   "pipeline_chunks": launches, "client_digests": bool(args.digests)},
        # per launch: algorithmic bytes of one launch / its average duration
        # (HIP events on the launch stream); the step's launches are equal
        "roofline": {"bound": "hbm", "achieved": achieved, "peak": HBM_PEAK_GBPS, "unit": "GB/s",
                     "frac": achieved / HBM_PEAK_GBPS,
                     "traffic": traffic, "traffic_detail": traffic_detail,
                     "kernel": f"{r['kernel']} (sa_fused_clients)" if r["fused"] else r["kernel"],
                     "kernel_ms_per_step": kern_ms,
                     "launches_per_step": launches,
                     "algorithmic_bytes_per_launch": bytes_alg / launches,
                     "kernel_ms_per_launch": kern_ms / launches,
                     "kernel_timing": r["kernel_timing"],
                     "valu": {"pcg64_draws_per_step": draws, "pair_draws_per_step": r["pair_draws"],
                              "one_sided_draws_per_step": r["one_sided_draws"],
                              "draws_per_s": draws / (kern_ms / 1e3),
                              "peak_pair_draws_per_s": pair_peak, "peak_one_sided_draws_per_s": one_peak,
                              "peak_source": ("measured on this rank's GPU before the bench touched it: "
                                              "tools/microbench/draw_issue 'dual pair28 E2' at 2 waves/SIMD and "
                                              "'dual one7 E2' at 8, median of 15 launches after 40 warm-up"
                                              if len(ceil) == 2 else
                                              "constants from profiles/r01/draw_issue_microbench.txt (another "
                                              "box): the same-box measurement failed"),
                              "ideal_ms_per_step": ideal_s * 1e3,
                              "frac": ideal_s / (kern_ms / 1e3),
                              "issue": int_ops}},
    }
    if rehearse:
        out["rehearsal"] = ("--rehearse-one-gpu: every rank on cuda:0; " + (
            "the product's NCCL process group and RcclComm with a distinct NCCL_HOSTID per rank, so RCCL runs its "
            "collectives between the ranks over its socket transport on lo (benchkit/standin.py one_gpu_rccl_comm)"
            if args.rehearse_comm == "rccl" else
            "collectives and their barriers through a shared host mapping (benchkit/standin.py)")
            + "; the N > 1 control flow, not the product's rate")
    out["cpu_baseline"] = cpu
    check_local = r.pop("check_local")
    out["check"] = {"round": 0, "decoded_digest": None, "note": CHECK_NOTE}
    if multi:
        out["designs_agree"] = True
        # the headline is in hand: from here on a failed or hung design (or
        # check) is recorded in the line and cannot cost it
        out["exchange"] = r["exchange"]
        # the exchange against the links: says by itself whether N is link- or kernel-bound
        out["roofline"]["exchange"] = r["exchange"].get("model")
        out["exchange_variants"] = [variant_summary(r)]
        if hasattr(comm, "info"):  # an RcclComm: what RCCL made of the run (every rank takes part)
            out["rccl"] = rccl_record(comm, rank, world, rccl_dir)
        out["variant_timeout_seconds"] = args.variant_timeout
        with wd.lock:
            wd.line = out if rank == 0 else {}
        settle_check(ctx, r, check_local, out, wd)
        run_variants(ctx, run_design, other_variants(args, head), variant_summary, out, wd, settle=combine_check)
        if args.host_resident_steps > 0 and head.name == "sharded" and not out.get("variants_incomplete"):
            run_contained(ctx, "host_resident", lambda: run_host_resident(
                ctx, args.host_resident_steps, min(3, args.warmup)), out, wd)
    else:
        out["check"]["decoded_digest"] = None if check_local is None else f"{check_local:016x}"
    if args.extra and world == 1:
        from sfl_amd import kernels as K

        kept = ctx["kept"]
        out["extra"] = extra_measurements(args, kept["xs"], kept["plan"], kept["gens"], K, torch, dev)
    wd.enter("done")
    if rank == 0:
        wd.emit(out)
    if out.get("variants_incomplete"):
        # a design failed on some ranks only: their peers' exchange may still
        # be pending on the GPU, which a communicator teardown would wait for
        sys.stdout.flush()
        sys.stderr.flush()
        os._exit(0)
    if comm is not None:
        comm.close()
        dist.destroy_process_group()


def rccl_record(comm, rank: int, world: int, log_dir) -> dict:
    """The line's ``rccl`` record (benchkit/rccl_log.py): this rank's RCCL
    init log and ``sa_comm_info``, gathered to every rank after the
    headline (its connections are set up by then)."""
    import shutil

    import torch.distributed as dist

    try:
        info = comm.info()
    except Exception as e:  # noqa: BLE001 - recorded, never costs the headline
        info = {"error": str(e)[:200]}
    mine = rccl_log.rank_summary(rank, log_dir, info)
    if log_dir and not os.environ.get("SFL_BENCH_RCCL_LOG_DIR"):
        shutil.rmtree(log_dir, ignore_errors=True)
    box = [None] * world
    dist.all_gather_object(box, mine)
    return rccl_log.combine(box, world)


def run_host_resident(ctx, steps: int, warmup: int) -> dict:
    """N > 1: the headline design with its inputs and results in pinned host
    memory (the north star's "starts and ends in host memory", in process):
    per step every local client's fp32 vector is copied H2D chunk by chunk on
    an H2D stream, chunk j is masked as soon as its copy lands, exchanged and
    decoded on the comm stream (the reduce-scatter sharded server), and this
    rank's decoded shard of chunk j goes D2H on a third stream; the next
    step's H2D of chunk j waits for that D2H (the decode buffer is reused)
    and for the previous launch of chunk j.  Timed like a design (barrier +
    synchronise on both sides, max over ranks).  Not `value`."""
    import torch
    import torch.distributed as dist

    from sfl_amd.parallel_sum import PipelinedMaskedSum, plan_generators, plan_rank, rank_shards

    args, world, rank, dev, comm = ctx["args"], ctx["world"], ctx["rank"], ctx["dev"], ctx["comm"]
    C, N = args.clients, args.elems
    plan = plan_rank(ctx["names"], world, rank)
    Lc = len(plan.clients)
    # one allocation per client (16-B aligned whatever N is), the headline's synthetic data
    host_x = [torch.empty(N, dtype=torch.float32).pin_memory() for _ in plan.clients]
    for i, c in enumerate(plan.clients):
        g = torch.Generator(device=dev).manual_seed(20260116 + c)
        host_x[i].copy_(torch.randn(N, generator=g, device=dev, dtype=torch.float32) * 1e-2)
    dev_x = [torch.empty(N, dtype=torch.float32, device=dev) for _ in plan.clients]
    pipe = PipelinedMaskedSum(comm, dev, N, args.chunks if args.chunks is not None else 8, exchange="sharded")
    sum_buf = torch.zeros(pipe.buffer_len, dtype=torch.int64, device=dev)
    dec = torch.zeros(pipe.buffer_len, dtype=torch.float64, device=dev)
    host_dec = torch.empty(pipe.buffer_len, dtype=torch.float64).pin_memory()
    shards = [(a, b) for a, b in rank_shards(pipe.bounds, world, rank, N)]
    total = warmup + steps
    gens = [[plan_generators(plan, pair_seed, offset=i * N + lo) for lo, _ in pipe.bounds] for i in range(total)]
    h2d, d2h = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    J = len(pipe.bounds)
    ev_in = [torch.cuda.Event() for _ in range(J)]
    ev_dec = [torch.cuda.Event() for _ in range(J)]
    ev_free = [torch.cuda.Event() for _ in range(J)]

    def after(j):  # comm stream current: chunk j exchanged and decoded
        a, b = shards[j]
        ev_dec[j].record(pipe.comm_stream)
        d2h.wait_event(ev_dec[j])
        with torch.cuda.stream(d2h):
            if b > a:
                host_dec[a:b].copy_(dec[a:b], non_blocking=True)
            ev_free[j].record(d2h)

    def step(i):
        with torch.cuda.stream(h2d):
            for j, (lo, hi) in enumerate(pipe.bounds):
                h2d.wait_event(ev_free[j])      # the previous step's D2H of this chunk's shard
                h2d.wait_event(pipe.events[j])  # the previous step's launch over this chunk
                for c in range(Lc):
                    dev_x[c][lo:hi].copy_(host_x[c][lo:hi], non_blocking=True)
                ev_in[j].record(h2d)
        pipe.run(dev_x, [1.0] * Lc, gens[i], plan.n_cross, sum_buf, None,
                 fxp_bits=args.fxp_bits, join=False, dec=dec, chunk_ready=ev_in, after_chunk=after)

    for i in range(warmup):
        step(i)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for i in range(steps):
        step(warmup + i)
    torch.cuda.synchronize()
    dist.barrier()
    torch.cuda.synchronize()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64)
    dist.all_reduce(el, op=dist.ReduceOp.MAX, group=control_group(ctx))
    ms = float(el[0]) * 1e3 / steps
    shard_elems = sum(b - a for a, b in shards)
    del host_x, dev_x, sum_buf, dec, host_dec, pipe, gens
    torch.cuda.empty_cache()
    return {"ms_per_step": ms, "grad_elems_per_s": C * N / (ms / 1e3), "steps": steps, "warmup": warmup,
            "pcie_bytes_per_rank_per_step": {"h2d": 4 * Lc * N, "d2h": 8 * shard_elems},
            "what": ("fp32 inputs in pinned host memory -> H2D per chunk (own stream) -> the headline's masking + "
                     "reduce-scatter + shard decode -> D2H of this rank's decoded shard (own stream); max over "
                     "ranks")}


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
        """Mean of ``reps`` calls after a warm one -- more calls for short ones
        (up to ~0.3 s of them, at most 20): config 2's 3.7 ms host round read
        8.8 ms once from 2 calls."""
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        fn()
        torch.cuda.synchronize()
        one = time.perf_counter() - t0
        reps = max(reps, min(20, int(0.3 / max(one, 1e-6))))
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
    host_x = torch.empty((C, N), dtype=torch.float32, pin_memory=True)  # [C, N] fp32, pinned once
    for c in range(C):
        host_x[c].copy_(xs[c])
    host_dec = torch.empty(N, dtype=torch.float64).pin_memory()
    # every client's masked vector back too: up to 16 GiB of pinned host
    # memory (config 3: 6.4 GB); config 5's 64 GB of wire images are left out
    images = 8 * C * N <= (16 << 30)
    host_m = torch.empty((C, N), dtype=torch.int64).pin_memory() if images else None
    dev_x = torch.empty((C, N), dtype=torch.float32, device=dev)
    dec = torch.empty(N, dtype=torch.float64, device=dev)
    s_h2d, s_cmp, s_d2h = torch.cuda.Stream(dev), torch.cuda.Stream(dev), torch.cuda.Stream(dev)
    # ~64 MB of inputs a chunk, 2..16 chunks (config 2's 160 MB in 16 chunks
    # spent its time in per-chunk host overhead: 10 ms against a 3.5 ms copy)
    bounds = chunk_bounds(N, max(2, min(16, (4 * C * N) // (64 << 20))))
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

    for with_images in ((False, True) if images else (False,)):
        t = timeit(lambda: host_round(with_images), reps=2)
        key = "host_resident_with_wire_images" if with_images else "host_resident"
        h2d, d2h = 4 * C * N, 8 * N + (8 * C * N if with_images else 0)
        res.update({f"{key}_ms": t * 1e3, f"{key}_grad_elems_per_s": C * N / t,
                    f"{key}_pcie_bytes": {"h2d": h2d, "d2h": d2h}})
    res["host_resident_note"] = ("pinned host fp32 inputs -> H2D -> fused quantize+mask+sum -> decode -> D2H of the "
                                 f"float64 aggregate (and of every client's masked u64 vector), {len(bounds)} chunks, "
                                 "H2D / compute / D2H on three streams" + ("" if images else
                                 "; no wire-image variant: 8*C*N bytes of pinned host memory exceed 16 GiB"))
    # the copy floor of the same bytes: the H2D of every client's input alone,
    # pinned, in the same chunks (the host-resident round cannot beat it)
    def h2d_only():
        with torch.cuda.stream(s_h2d):
            for lo, hi in bounds:
                for c in range(C):
                    dev_x[c, lo:hi].copy_(host_x[c, lo:hi], non_blocking=True)

    t = timeit(h2d_only, reps=2)
    res.update({"h2d_floor_ms": t * 1e3, "h2d_floor_GBps": 4 * C * N / t / 1e9,
                "host_resident_vs_h2d_floor": t / (res["host_resident_ms"] / 1e3)})
    if not images:
        return res

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
