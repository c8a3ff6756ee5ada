"""One process per GPU: simulated clients sharded across ranks, the masked
partial sums reduced to the server rank with RCCL over xGMI.

North-star layout (BASELINE.json): C clients over W GPUs, clients assigned in
contiguous blocks (rank r owns clients [r*C/W, (r+1)*C/W)).  Each rank runs
ONE fused launch (``sa_fused_clients``) over its L = C/W local clients:
internal pair streams are expanded once and applied to both clients, each
local client additionally applies its C - L cross-rank streams (the peer's
half of those pairs runs on the peer's rank).  The only exchange is the
uint64 masked partial sum: reduce-scattered so that every rank is the
server of one shard and decodes it (``sa_comm_reduce_scatter_u64``, the
bench's headline design, optionally followed by a float64 gather to the
root), or reduced to rank 0 by ``ncclReduce`` (``sa_comm_reduce_u64``) —
bit-exact for any RCCL algorithm because uint64 addition is associative
mod 2^64.  This replaces the RayFed ``.to(server)`` transfer plus the
server ``np.sum`` (sfl/distributed/op_strategy.py:131-141,
sfl/security/aggregation/sparse_plain_aggregator.py:86-94).

The shard planning here is pure host logic (tested with gloo on CPU); the
data path is the HIP kernels plus RCCL.
"""

from __future__ import annotations

import ctypes as C
from dataclasses import dataclass, field

from . import _lib as L


def client_shard(n_clients: int, world: int, rank: int) -> list[int]:
    """Contiguous block of client indices owned by ``rank``."""
    if n_clients % world:
        raise ValueError(f"{n_clients} clients do not split evenly over {world} ranks")
    per = n_clients // world
    return list(range(rank * per, (rank + 1) * per))


@dataclass
class LocalPlan:
    """What one rank launches: pair streams among its clients, cross streams
    to clients on other ranks (client-major, equal count per client)."""

    clients: list[int]
    pairs: list[tuple[int, int]] = field(default_factory=list)         # (u, v) global ids, u < v local
    pair_signs: list[int] = field(default_factory=list)                # sign for u
    cross: list[tuple[int, int, int]] = field(default_factory=list)    # (client, peer, sign)

    @property
    def n_cross(self) -> int:
        return len(self.cross) // max(1, len(self.clients))


def plan_rank(names: list[str], world: int, rank: int) -> LocalPlan:
    """Streams rank ``rank`` must expand.  Signs follow the reference's
    ``party > self._party`` name rule (secure_aggregation.ipynb cell 15)."""
    C = len(names)
    mine = client_shard(C, world, rank)
    p = LocalPlan(clients=mine)
    for i, u in enumerate(mine):
        for v in mine[i + 1:]:
            p.pairs.append((u, v))
            p.pair_signs.append(1 if names[v] > names[u] else -1)
    local = set(mine)
    for u in mine:
        for v in range(C):
            if v not in local:
                p.cross.append((u, v, 1 if names[v] > names[u] else -1))
    return p


def plan_generators(plan: LocalPlan, seed_of, offset: int = 0):
    """(pair_gens, pair_signs, cross_streams) for ``kernels.fused_clients``.
    ``seed_of(u, v)`` returns the pairwise seed (symmetric)."""
    pg = [L.pcg64_advance(L.pcg64_from_seed(seed_of(u, v)), offset) for (u, v) in plan.pairs]
    cross = [(L.pcg64_advance(L.pcg64_from_seed(seed_of(u, v)), offset), s, v) for (u, v, s) in plan.cross]
    return pg, list(plan.pair_signs), cross


class RcclComm:
    """Our own RCCL communicator (C-ABI ``sa_comm_*``), rendezvoused through
    an existing torch.distributed group (which only carries the unique id)."""

    def __init__(self, rank: int, world: int, device: int, group=None):
        import torch.distributed as dist

        uid = (C.c_char * L.SA_UNIQUE_ID_BYTES)()
        if rank == 0:
            L.check(L.lib().sa_comm_unique_id(uid, L.SA_UNIQUE_ID_BYTES), "sa_comm_unique_id")
        box = [bytes(uid) if rank == 0 else None]
        dist.broadcast_object_list(box, src=0, group=group)
        uid = (C.c_char * L.SA_UNIQUE_ID_BYTES).from_buffer_copy(box[0])
        h = C.c_void_p()
        L.check(L.lib().sa_comm_init(C.byref(h), uid, world, rank, device), "sa_comm_init")
        self._h = h
        self.rank, self.world = rank, world

    def reduce_u64(self, send, recv, root: int = 0):
        import torch

        stream = torch.cuda.current_stream(send.device).cuda_stream
        L.check(L.lib().sa_comm_reduce_u64(self._h, C.c_void_p(send.data_ptr()),
                                           C.c_void_p(recv.data_ptr()) if recv is not None else None,
                                           send.numel(), root, C.c_void_p(stream)), "sa_comm_reduce_u64")
        return recv

    def allreduce_u64(self, send, recv):
        import torch

        stream = torch.cuda.current_stream(send.device).cuda_stream
        L.check(L.lib().sa_comm_allreduce_u64(self._h, C.c_void_p(send.data_ptr()), C.c_void_p(recv.data_ptr()),
                                              send.numel(), C.c_void_p(stream)), "sa_comm_allreduce_u64")
        return recv

    def reduce_scatter_u64(self, send, recv):
        """``recv`` (rank r) = the masked sum of ``send``'s r-th of ``world``
        equal shards (in place when ``recv`` is that shard of ``send``)."""
        import torch

        if send.numel() != recv.numel() * self.world:
            raise ValueError(f"reduce_scatter: {send.numel()} elements do not split into {self.world} x {recv.numel()}")
        stream = torch.cuda.current_stream(send.device).cuda_stream
        L.check(L.lib().sa_comm_reduce_scatter_u64(self._h, C.c_void_p(send.data_ptr()), C.c_void_p(recv.data_ptr()),
                                                   recv.numel(), C.c_void_p(stream)), "sa_comm_reduce_scatter_u64")
        return recv

    def alltoall_u64(self, send, recv):
        """For every rank p != this one: ``recv``'s p-th of ``world`` equal
        slots = rank p's shard (this rank's slot) of ``send``; this rank's own
        slot of ``recv`` is not written (its shard stays in ``send``)."""
        import torch

        if send.numel() != recv.numel() or send.numel() % self.world:
            raise ValueError(f"alltoall: {send.numel()} / {recv.numel()} elements do not split into {self.world} slots")
        stream = torch.cuda.current_stream(send.device).cuda_stream
        L.check(L.lib().sa_comm_alltoall_u64(self._h, C.c_void_p(send.data_ptr()), C.c_void_p(recv.data_ptr()),
                                             send.numel() // self.world, C.c_void_p(stream)), "sa_comm_alltoall_u64")
        return recv

    def gather_f64(self, send, recv, root: int = 0):
        """Root's ``recv`` (``world`` x ``send.numel()``) = every rank's float64 shard in rank order."""
        import torch

        if self.rank == root and (recv is None or recv.numel() != send.numel() * self.world):
            raise ValueError("gather: the root needs a receive buffer of world x shard elements")
        stream = torch.cuda.current_stream(send.device).cuda_stream
        L.check(L.lib().sa_comm_gather_f64(self._h, C.c_void_p(send.data_ptr()),
                                           C.c_void_p(recv.data_ptr()) if recv is not None else None,
                                           send.numel(), root, C.c_void_p(stream)), "sa_comm_gather_f64")
        return recv

    def info(self) -> dict:
        """What RCCL made of this communicator: {"nranks", "rank", "device"}
        (ncclCommCount / ncclCommUserRank / ncclCommCuDevice)."""
        n, r, d = C.c_int(-1), C.c_int(-1), C.c_int(-1)
        L.check(L.lib().sa_comm_info(self._h, C.byref(n), C.byref(r), C.byref(d)), "sa_comm_info")
        return {"nranks": n.value, "rank": r.value, "device": d.value}

    def close(self):
        if self._h:
            L.check(L.lib().sa_comm_destroy(self._h), "sa_comm_destroy")
            self._h = None


def chunk_bounds(n: int, chunks: int, align: int = 1024) -> list[tuple[int, int]]:
    """Split [0, n) into ``chunks`` ranges whose starts are multiples of
    ``align`` elements (keeps every chunk's buffers 16-B aligned)."""
    chunks = max(1, chunks)
    step = -(-n // chunks)
    step = -(-step // align) * align
    out = []
    lo = 0
    while lo < n:
        out.append((lo, min(n, lo + step)))
        lo += step
    return out or [(0, 0)]


def shard_layout(bounds: list[tuple[int, int]], world: int) -> list[tuple[int, int]]:
    """The sharded server's split of every pipeline chunk:
    chunk [lo, hi) is reduce-scattered as ``world`` equal shards of ``k``
    elements (``(hi - lo) / world`` rounded up to a multiple of 128, so every
    shard starts 1 KiB aligned), rank r's shard starting at ``lo + r*k``.
    Returns [(lo, k)] per chunk.  Only the last chunk may need padding (the
    pipeline's chunk starts are multiples of ``1024 * world``), so its shards
    may run past n: buffers hold ``padded_len`` elements."""
    return [(lo, -(-(hi - lo) // (world * 128)) * 128) for lo, hi in bounds]


def padded_len(bounds: list[tuple[int, int]], world: int) -> int:
    """Elements a sharded-server buffer must hold (n plus < world of padding)."""
    return max((lo + world * k for lo, k in shard_layout(bounds, world)), default=0)


def rank_shards(bounds: list[tuple[int, int]], world: int, rank: int, n: int) -> list[tuple[int, int]]:
    """The element ranges [a, b) of [0, n) whose masked sum rank ``rank``
    receives (and decodes) as the sharded server, one per chunk."""
    out = []
    for lo, k in shard_layout(bounds, world):
        a = min(n, lo + rank * k)
        out.append((a, min(n, a + k)))
    return out


def element_shard(n: int, world: int, rank: int) -> tuple[int, int, int]:
    """Element sharding (SURVEY.md §8(e)'s alternative to client sharding):
    rank ``rank`` masks elements [e0, e0 + n_loc) of EVERY client, each pair
    stream jumped e0 draws ahead (``plan_generators(..., offset=round + e0)``),
    so its slice of the masked sum is complete without any exchange.  Slices
    are ``k`` elements (n / world rounded up to 128; the last one shorter or
    empty), so a gather moves equal counts.  Returns (e0, n_loc, k)."""
    k = shard_layout([(0, n)], world)[0][1]
    e0 = min(n, rank * k)
    return e0, min(n, e0 + k) - e0, k


class PipelinedMaskedSum:
    """One rank's share of a secure-aggregation round with the exchange
    overlapped: the fused masking launch of chunk j (compute stream) runs
    while chunk j-1's uint64 partial sum is reduced to the server rank
    (``ncclReduce`` on a separate comm stream, ordered by an event per
    chunk).  Chunk j's streams start ``lo_j`` draws into the round, so the
    result is bit-identical to one launch over the whole vector.

    ``chunk_gens[j]`` = ``plan_generators(plan, seed_of, offset=round_offset + lo_j)``.

    ``exchange="sharded"``: the sharded server of SURVEY.md §8(e) instead of
    the reduce to one rank -- each chunk's partial sum is reduce-scattered in
    place (rank r receives the masked sum of its shard, ``shard_layout``),
    every rank decodes its shard into ``dec`` on the comm stream, and with
    ``gather=True`` the float64 shards are gathered into the root's ``dec``.
    ``exchange="direct"``: the same sharded server with the reduce-scatter
    done as direct shard transfers (``alltoall_u64``: each shard crosses one
    link into a staging buffer) and a local ``sum_u64`` of the ``world``
    shards into this rank's shard of the partial sum.
    Partial-sum and ``dec`` buffers hold ``self.buffer_len`` elements (n plus
    < world of padding that is reduced and decoded but never read)."""

    def __init__(self, comm: RcclComm | None, device, n: int, chunks: int, exchange: str = "reduce"):
        import torch

        if exchange not in ("reduce", "sharded", "direct"):
            raise ValueError(f"exchange must be 'reduce', 'sharded' or 'direct', not {exchange!r}")
        if exchange != "reduce" and comm is None:
            raise ValueError("the sharded server needs a communicator")
        self.comm = comm
        self.device = device
        self.n = n
        self.exchange = exchange
        world = comm.world if comm is not None else 1
        # sharded: chunk starts on multiples of 1024 * world, so only the last
        # chunk's shards can run past its end (into padding, never into the
        # next chunk that the compute stream may be masking)
        sharded = exchange != "reduce"
        self.bounds = chunk_bounds(n, chunks, align=1024 * world if sharded else 1024)
        self.shards = shard_layout(self.bounds, world) if sharded else None
        self.buffer_len = padded_len(self.bounds, world) if sharded else n
        # direct: the other ranks' shards of one chunk land here (the comm
        # stream runs one chunk's exchange at a time, so one chunk's worth)
        self.staging = (torch.empty(world * max(k for _, k in self.shards), dtype=torch.int64, device=device)
                        if exchange == "direct" and world > 1 else None)
        self.comm_stream = torch.cuda.Stream(device) if comm is not None else None
        self.events = [torch.cuda.Event() for _ in self.bounds]
        # reduce of chunk j done (comm stream): the next round's chunk-j launch
        # waits for it, and for nothing else of the previous round
        self.reduced = [torch.cuda.Event() for _ in self.bounds]
        self._pending = [False] * len(self.bounds)

    def run(self, xs, weights, chunk_gens, n_cross: int, sum_buf, recv=None, *, root: int = 0,
            fxp_bits: int = 18, digests=None, flags=None, kernel_events: list | None = None,
            exchange_events: list | None = None, join: bool = True, dec=None, divisor: float = 1.0,
            gather: bool = False, chunk_ready: list | None = None, after_chunk=None):
        """``kernel_events``: if given, a timing-event pair recorded around
        each chunk's masking launch is appended (kernel time without the
        exchange); ``exchange_events`` likewise around each chunk's reduce on
        the comm stream (from the moment that chunk's launch has finished
        here, so the wait for slower peers counts).  ``join=False`` leaves the last reduces running on the
        comm stream (the caller synchronises the device before reading the
        result); a following run() still orders each chunk's launch after
        that chunk's previous reduce, so back-to-back rounds overlap one
        round's exchange tail with the next round's first launches.

        Host-resident pipelines (bench.py's host_resident): ``chunk_ready[j]``
        is an event the compute stream waits for before chunk j's launch
        (its H2D), and ``after_chunk(j)`` is called with the comm stream
        current right after chunk j's exchange and decode (to enqueue its
        D2H)."""
        import torch

        from . import kernels as K

        if len(chunk_gens) != len(self.bounds):
            raise ValueError(f"{len(chunk_gens)} generator sets for {len(self.bounds)} chunks")
        sharded = self.exchange != "reduce"
        if sharded:
            if recv is not None:
                raise ValueError("the sharded server reduces in place (recv=None)")
            if dec is None or dec.numel() < self.buffer_len or sum_buf.numel() < self.buffer_len:
                raise ValueError(f"sharded server: sum_buf and dec need {self.buffer_len} elements")
        compute = torch.cuda.current_stream(self.device)
        for j, (lo, hi) in enumerate(self.bounds):
            pg, ps, cross = chunk_gens[j]
            if self._pending[j]:  # the previous round's reduce of this chunk still reads sum_buf
                compute.wait_event(self.reduced[j])
                self._pending[j] = False
            if chunk_ready is not None:
                compute.wait_event(chunk_ready[j])
            if kernel_events is not None:
                kernel_events.append((torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)))
                kernel_events[-1][0].record(compute)
            K.fused_clients([x[lo:hi] for x in xs], weights, pg, ps, cross, n_cross, sum_buf[lo:hi],
                            fxp_bits=fxp_bits, digests=digests, flags=flags)
            if kernel_events is not None:
                kernel_events[-1][1].record(compute)
            if self.comm is not None:
                self.events[j].record(compute)
                self.comm_stream.wait_event(self.events[j])
                with torch.cuda.stream(self.comm_stream):
                    if exchange_events is not None:
                        exchange_events.append((torch.cuda.Event(enable_timing=True),
                                                torch.cuda.Event(enable_timing=True)))
                        exchange_events[-1][0].record(self.comm_stream)
                    if sharded:
                        lo_s, k = self.shards[j]
                        W, r = self.comm.world, self.comm.rank
                        mine = lo_s + r * k
                        shard = sum_buf[mine:mine + k]
                        if self.exchange == "sharded":
                            self.comm.reduce_scatter_u64(sum_buf[lo_s:lo_s + k * W], shard)
                        elif W > 1:  # direct: own shard first (sum_u64's out may alias in[0])
                            st = self.staging[:k * W]
                            self.comm.alltoall_u64(sum_buf[lo_s:lo_s + k * W], st)
                            K.sum_u64([shard] + [st[p * k:(p + 1) * k] for p in range(W) if p != r], shard)
                        K.decode(shard, dec[mine:mine + k], fxp_bits=fxp_bits, divisor=divisor)
                        if gather:
                            self.comm.gather_f64(dec[mine:mine + k], dec[lo_s:lo_s + k * self.comm.world]
                                                 if self.comm.rank == root else None, root=root)
                    else:
                        self.comm.reduce_u64(sum_buf[lo:hi], recv[lo:hi] if recv is not None else None,
                                             root=root)
                    if after_chunk is not None:
                        after_chunk(j)
                    if exchange_events is not None:
                        exchange_events[-1][1].record(self.comm_stream)
                    self.reduced[j].record(self.comm_stream)
                self._pending[j] = True
        if self.comm is not None and join:
            compute.wait_stream(self.comm_stream)
            self._pending = [False] * len(self.bounds)
        if sharded:
            return dec
        return recv if recv is not None else sum_buf
