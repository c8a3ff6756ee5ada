"""The secure aggregation split at the party boundary: what runs inside each
participant's process and what runs inside the server's.

The reference's ``SecureAggregator`` (un-vendored ``secretflow-lite``) keeps
one ``_Masker`` per participant on that participant's own device; only DH
public keys reach the driver, and only masked vectors leave a client
(``docs/developer/algorithm/secure_aggregation.ipynb:227-239``: "each
participant outputs" ``y_u``; ``sfl/security/aggregation/sparse_plain_aggregator.py:86``:
``data = [d.to(self.device) for d in data]``).  The functions below are those
per-device steps, written so a secretflow device can run them remotely:

* every argument and result is a plain picklable value (a :class:`Masker`,
  host arrays, a :class:`MaskedPayload`);
* the masker is threaded through functionally -- ``mask_payload`` returns
  the advanced masker as a second result (``num_returns=2``) -- so the
  generator positions persist across rounds in the party's object store
  without an actor and without the driver ever holding the state;
* per-element work runs on the party's GPU through ``libsfl_sa`` (``sa_mask``
  on the client, ``sa_sum_u64`` + ``sa_decode`` on the server); numpy's
  rejection of a raw PCG64 0 is resolved on the client before its vector
  leaves (``sa_pcg64_find_zero`` / ``sa_stream_shift``), as the reference's
  ``Generator.integers`` does inside ``_Masker``.

``sfl_amd.compat.secretflow.SecureAggregator`` drives these through
secretflow-shaped devices; ``tests/test_compat_secretflow.py`` runs them in a
spawned process per party.
"""

from __future__ import annotations

import os
import threading
from dataclasses import dataclass, field

import numpy as np

from .masker import Masker

_F32, _F64, _I64 = np.dtype(np.float32), np.dtype(np.float64), np.dtype(np.int64)


# the server's large sum_decode stages vectors that are not pooled results
# (vectors deserialised from other processes) through the feeder; with
# SFL_SERVER_REGISTER=1 it registers them lazily instead: 125-129 against
# 121-123 ms at 8 x 100M (tools/archive/server_register_ab.sh)
SERVER_REGISTER = os.environ.get("SFL_SERVER_REGISTER", "0") == "1"


@dataclass
class MaskedPayload:
    """One client's masked contribution: what crosses the wire to the server.

    ``u64`` is every layer's masked uint64 vector packed in layer order (the
    reference ships the per-layer arrays; the packing is the same elements
    with one header).  ``digest`` is the XOR of its 64-bit words, checked by
    the server after the transfer."""
    party: str
    u64: np.ndarray
    sizes: list
    shapes: list
    container: str          # "array" | "list" | "tuple"
    as_torch: bool
    digest: int
    fxp_bits: int
    positions: dict = field(default_factory=dict)  # peer -> stream position the round started at


# large host payloads run chunked through three streams (_mask_vector_pipelined,
# _sum_decode_pipelined); False restores the one-shot copies (tools/party_bench.py A/B)
LARGE_PIPELINE = True

# scratch of the blocking small-call library entries (sa_mask_host,
# sa_sum_decode_host), per GPU of this process, grown to the largest call
_SCRATCH: dict = {}
_SCRATCH_LOCK = threading.Lock()


def _scratch(gpu: int, pin_bytes: int, dev_bytes: int):
    import torch

    cur = _SCRATCH.get(gpu)
    if cur is None or cur[0].numel() < pin_bytes or cur[1].numel() < dev_bytes:
        pb = max(pin_bytes, cur[0].numel() if cur else 0)
        db = max(dev_bytes, cur[1].numel() if cur else 0)
        cur = (torch.empty(pb, dtype=torch.uint8, pin_memory=True),
               torch.empty(db, dtype=torch.uint8, device=torch.device("cuda", gpu)))
        _SCRATCH[gpu] = cur
    return cur


# --------------------------------------------------------------- key set-up
def new_masker(party: str, fxp_bits: int = 18) -> Masker:
    """Runs on the participant: a fresh DH key pair (its private half never
    leaves this process)."""
    return Masker(str(party), int(fxp_bits))


def public_key(masker: Masker) -> int:
    """Runs on the participant: the only value of its masker the driver sees."""
    return int(masker.public_key)


def agree(masker: Masker, peer_keys: dict, seeds: dict | None = None) -> Masker:
    """Runs on the participant: pairwise seeds from the revealed public keys
    (``seeds``: explicit ``{peer: seed | (state, inc)}`` for tests).  Returns
    the agreed masker (a new object, like ``mask_payload``)."""
    masker = masker.copy()
    if seeds is None:
        masker.agree({str(k): int(v) for k, v in peer_keys.items()})
    else:
        for peer in peer_keys:
            if peer == masker.party:
                continue
            s = seeds[peer]
            if isinstance(s, (tuple, list)):
                masker.set_state(peer, *s)
            else:
                masker.set_seed(peer, int(s))
    return masker


# ------------------------------------------------------------- client side
def _layers(payload):
    if isinstance(payload, tuple):
        return list(payload), "tuple"
    if isinstance(payload, list):
        return list(payload), "list"
    return [payload], "array"


def _host_weight(w):
    if w is None:
        return None
    try:
        import torch

        if isinstance(w, torch.Tensor):
            from ... import hostpipe as H

            return w.detach().numpy() if w.device.type == "cpu" else H.d2h(w, pooled=False)
    except ImportError:  # pragma: no cover
        pass
    return w


def mask_payload(masker: Masker, payload, weight=None, gpu: int | None = 0):
    """Runs on the participant: quantize ``payload * weight`` and add the
    pairwise masks (``sa_mask`` on this party's GPU ``gpu``).

    Returns ``(MaskedPayload, masker)``, a NEW masker advanced past this
    round's draws (numpy's rejections included); the one passed in is left
    as it was -- an object store hands the function a copy anyway, and an
    in-process device must not see a round that failed part-way advance
    some parties' streams."""
    from .secure_aggregator import _compute_dtype, _np_dtype, _shape

    masker = masker.copy()
    layers, container = _layers(payload)
    weight = _host_weight(weight)
    shapes = [_shape(a) for a in layers]
    sizes = [int(np.prod(sh)) if sh else 1 for sh in shapes]
    as_torch = _is_torch(layers[0]) if layers else False
    plan = []
    for a, sh in zip(layers, shapes):
        ldt = _np_dtype(a)
        ct = _compute_dtype(ldt, weight, masker.fxp_bits)
        if ct not in (_F32, _F64, _I64):
            raise NotImplementedError(f"arithmetic type {ct} (data {ldt}) is not supported")
        if ldt.kind in "biu" and ldt != _I64 and ct.kind == "i":
            raise NotImplementedError(f"integer data of type {ldt} is not supported")
        xt = ldt if ldt in (_F32, _F64, _I64) else (_I64 if ldt.kind in "biu" else _F64)
        wvec = None
        if weight is not None and np.ndim(weight):
            wvec = np.ascontiguousarray(np.broadcast_to(np.asarray(weight), sh).astype(ct)).reshape(-1)
        plan.append((xt, ct, wvec))

    # consecutive layers draw consecutive stream positions (the reference's
    # per-layer rng.integers calls): layers of one element / arithmetic type
    # under a scalar weight are masked as ONE vector -- bit-identical
    groups, cur = [], None
    for li, (xt, ct, wvec) in enumerate(plan):
        key = (xt, ct)
        if cur is not None and cur[0] == key and wvec is None and cur[2] is None:
            cur[1].append(li)
        else:
            cur = [key, [li], wvec]
            groups.append(cur)

    start = {p: masker.position(p) for p in masker.peers}
    bounds = np.cumsum([0] + sizes)
    out, digest = None, 0
    for (xt, ct), lis, wvec in groups:
        lo, hi = int(bounds[lis[0]]), int(bounds[lis[-1] + 1])
        if hi == lo:
            continue
        xs = [layers[li] for li in lis]
        wscalar = 1.0
        if weight is not None and not np.ndim(weight):
            wscalar = float(weight) if ct.kind == "f" else int(weight)
        vec, extra, dig = _mask_vector(masker, xs, xt, ct, wscalar, wvec, gpu)
        if out is None and lo == 0 and hi == bounds[-1]:
            out = vec  # one group: its (fresh) vector is the payload, no copy
        else:
            if out is None:
                out = np.empty(int(bounds[-1]), dtype=np.uint64)
            out[lo:hi] = vec
        # the XOR digest of the whole payload is the XOR of the groups' digests
        digest ^= dig if dig is not None else (int(np.bitwise_xor.reduce(vec)) if vec.size else 0)
        masker.consume(hi - lo)
        for peer, k in extra.items():
            masker.skip(peer, k)
    if out is None:
        out = np.zeros(int(bounds[-1]), dtype=np.uint64)
    return (MaskedPayload(masker.party, out, sizes, shapes, container, as_torch, digest, masker.fxp_bits, start),
            masker)


def _is_cuda(a) -> bool:
    return _is_torch(a) and a.device.type != "cpu"


def _is_torch(a) -> bool:
    try:
        import torch

        return isinstance(a, torch.Tensor)
    except ImportError:  # pragma: no cover
        return False


def _mask_vector(masker: Masker, xs: list, xt: np.dtype, ct: np.dtype, wscalar, wvec, gpu):
    """One launch group on the party's GPU: ``sa_mask`` over the packed
    layers ``xs`` from the masker's current stream positions; a flagged raw
    0 is moved onto numpy's stream (``sa_stream_shift``).  Returns the host
    uint64 vector, ``{peer: extra raw draws}`` and its XOR digest when the
    device formed it (None: the caller XORs the host vector).  Large host
    layers take ``_mask_vector_pipelined``.

    The masked vector and the PRG flag word share one device buffer, so a
    small call (up to ``SMALL_CALL_BYTES``) brings both back with one copy
    into pinned memory and one synchronisation."""
    import torch

    from ... import _lib as L
    from ... import hostpipe as H
    from ... import kernels as K
    from .secure_aggregator import SMALL_CALL_BYTES

    if gpu is None:
        raise RuntimeError("the party has no GPU: libsfl_sa masks on the device")
    dev = torch.device("cuda", gpu)
    tdt = {_F32: torch.float32, _F64: torch.float64, _I64: torch.int64}
    n = int(sum(int(np.prod(_shape_of(a))) for a in xs))
    small = 8 * n <= SMALL_CALL_BYTES
    streams = masker.streams()
    if all(not isinstance(a, torch.Tensor) or a.device.type == "cpu" for a in xs):
        # CPU tensors (``get_weights()``'s state-dict values) are host layers:
        # their numpy views, no copy
        xs = [a.detach().numpy() if isinstance(a, torch.Tensor) else a for a in xs]
    host_layers = not any(isinstance(a, torch.Tensor) for a in xs)
    if not small and wvec is None and host_layers and LARGE_PIPELINE:
        # host layers of a large payload: chunked H2D / mask / D2H overlap
        got = _mask_vector_pipelined(masker, xs, xt, ct, wscalar, gpu)
        if got is not None:
            return got
        # numpy's rejection of a raw 0: the device path below re-positions the streams
    if small and wvec is None and host_layers:
        # host layers of a small payload: ONE blocking library call
        flat = (np.asarray(xs[0], dtype=xt).reshape(-1) if len(xs) == 1 else
                np.concatenate([np.asarray(a, dtype=xt).reshape(-1) for a in xs]))
        with _SCRATCH_LOCK, torch.cuda.device(dev):
            pin, dbuf = _scratch(gpu, *K.mask_host_scratch(n, xt.itemsize))
            host, flag = K.mask_host(flat, ct, streams, pin, dbuf, weight=wscalar, fxp_bits=masker.fxp_bits)
        if not flag & L.SA_FLAG_PRG_REJECT:
            return host, {}, None
        # numpy's rejection of a raw 0 (p = 2^-64 a draw): the device path below re-positions the streams
    with torch.cuda.device(dev):
        if not any(isinstance(a, torch.Tensor) for a in xs):
            # host layers (FedAvgW's get_weights payloads): packed on the host, ONE H2D copy
            if small:
                pin = torch.empty(n, dtype=tdt[xt], pin_memory=True)
                pv = pin.numpy()
                off = 0
                for a in xs:
                    a = np.asarray(a).reshape(-1)
                    pv[off:off + a.size] = a
                    off += a.size
                x = pin.to(dev, non_blocking=True)
            else:
                flat = (np.ascontiguousarray(np.asarray(xs[0]), dtype=xt).reshape(-1) if len(xs) == 1 else
                        np.concatenate([np.asarray(a, dtype=xt).reshape(-1) for a in xs]))
                x = H.h2d(flat, dev)
        else:
            # device tensors as they are; CPU tensors cast on the host (no DMA), then pinned H2D
            parts = [a.detach().reshape(-1).to(device=dev, dtype=tdt[xt]) if _is_cuda(a) else
                     H.h2d(a.detach().reshape(-1).to(tdt[xt]) if _is_torch(a) else
                           np.ascontiguousarray(np.asarray(a), dtype=xt).reshape(-1), dev)
                     for a in xs]
            x = parts[0] if len(parts) == 1 else torch.cat(parts)
        x = x.contiguous()
        if x.data_ptr() % 16:
            x = x.clone()
        wv = None if wvec is None else H.h2d(wvec, dev)
        buf = torch.empty(n + 1, dtype=K.U64, device=dev)  # masked vector | flag word
        out = buf[:n]
        flags = buf[n:].view(torch.int32)[:1]
        buf[n:].zero_()
        K.mask(x, out, streams, weight=wscalar, weight_vec=wv, compute_dtype=tdt[ct],
               fxp_bits=masker.fxp_bits, flags=flags)
        if small:
            pin_out = torch.empty(n + 1, dtype=K.U64, pin_memory=True)
            pin_out.copy_(buf, non_blocking=True)
            torch.cuda.current_stream(dev).synchronize()
            hv = pin_out.numpy().view(np.uint64)
            flag = int(hv[n]) & 0xFFFFFFFF  # the flag word's low half (little-endian)
        else:
            flag = int(flags.item())
        extra = {}
        if flag & L.SA_FLAG_PRG_REJECT:
            found = K.rejected_draws_many([g for g, _, _ in streams], n, dev)
            for peer, (gen, sign, _), (pts, total) in zip(masker.peers, streams, found):
                for k, shift in pts:
                    K.stream_shift(out, gen, sign, k, shift)
                if total > n:
                    extra[peer] = total - n
            host = H.d2h(out).view(np.uint64)
        elif small:
            host = hv[:n].copy()
        else:
            host = H.d2h(out).view(np.uint64)
    return host, extra, None


def _mask_vector_pipelined(masker: Masker, xs: list, xt: np.dtype, ct: np.dtype, wscalar, gpu):
    """A large launch group from host layers, chunked through three streams
    (``sfl_amd/hostpipe.py``): chunk j's H2D straight from the caller's
    layers (registered for the call, else staged through pinned slots by a
    feeder thread), its ``sa_mask``
    at stream offset ``lo`` (the XOR digest accumulated on the device), its
    D2H into the result -- a recycled registered buffer, or a fresh array
    reached through a pinned slot -- the copies of different chunks
    overlapping each other.
    Bit-identical to one launch over the whole group (chunk j draws
    positions [lo, hi) of every stream).  Returns (host uint64 vector, {},
    digest), or None when the round drew a raw 0 (numpy's rejection: the
    caller's device path replays it from the same positions)."""
    import torch

    from ... import _lib as L
    from ... import hostpipe as H
    from ... import kernels as K

    dev = torch.device("cuda", gpu)
    tdt = {_F32: torch.float32, _F64: torch.float64, _I64: torch.int64}
    ph = H.Phases("mask_payload")
    layers = H.host_layers(xs, xt)
    n = int(sum(a.size for a in layers))
    bounds = H.page_bounds(H.chunk_bounds(n, target=16), [layers])
    out = H.FreshOutput(n, np.uint64, bounds)  # its pages start faulting in now
    s_in, s_k, s_out = H.streams(dev)
    with torch.cuda.device(dev), H.Pinned(layers) as pin:
        cur = torch.cuda.current_stream(dev)
        x = torch.empty(n, dtype=tdt[xt], device=dev)
        buf = torch.empty(n + 2, dtype=K.U64, device=dev)  # masked vector | digest | flag word
        res, dig, flags = buf[:n], buf[n:n + 1], buf[n + 1:].view(torch.int32)[:1]
        buf[n:].zero_()
        ready = torch.cuda.Event()
        ready.record(cur)
        s_in.wait_event(ready)
        s_k.wait_event(ready)
        copies = [[(x[lo:hi], H.pieces(layers, lo, hi))] for lo, hi in bounds]
        # registered layers: every H2D issued at once, async; else staged by the feeder
        feed = H.Issued(s_in, copies, pin) if pin.ok else H.Feeder(s_in, copies)
        try:
            def launch(j):
                lo, hi = bounds[j]
                e_k = torch.cuda.Event()
                with torch.cuda.stream(s_k):
                    s_k.wait_event(feed.ready(j))
                    K.mask(x[lo:hi], res[lo:hi], masker.streams(offset=lo), weight=wscalar,
                           compute_dtype=tdt[ct], fxp_bits=masker.fxp_bits, digest=dig, flags=flags)
                    e_k.record(s_k)
                return e_k

            def d2h(j, e_k):
                lo, hi = bounds[j]
                out.copy_in(j, res[lo:hi], s_out, e_k)

            for j in range(len(bounds)):  # chunk j launches once the feeder has issued its copy in
                d2h(j, launch(j))
            meta = torch.empty(2, dtype=K.U64, pin_memory=True)
            with torch.cuda.stream(s_k):
                meta.copy_(buf[n:], non_blocking=True)
            ph.mark("pipeline")
        finally:
            feed.join(check=False)  # the feeder is done with the inputs
            out.close()
            s_k.synchronize()
            s_out.synchronize()
            s_in.synchronize()
            cur.wait_stream(s_k)  # x / buf were allocated on the current stream
        feed.join()
        ph.mark("wait")
    ph.note(pinned=pin.ok, **pin.stats, **out.stats)
    ph.done()
    digest, flag = int(meta[0]) & ((1 << 64) - 1), int(meta[1]) & 0xFFFFFFFF
    if flag & L.SA_FLAG_PRG_REJECT:
        return None
    return out.array, {}, digest


def _shape_of(a):
    return tuple(a.shape) if hasattr(a, "shape") else np.shape(a)


# ------------------------------------------------------------- server side
def sum_decode(*payloads: MaskedPayload, weights=None, average: bool = False, gpu: int | None = 0):
    """Runs on the server: check each payload's digest, sum the masked
    vectors mod 2^64 (the masks cancel) and decode ``int64(S) / 2^fxp`` as
    float64, divided by C or ``sum(weights)`` (element-wise for per-element
    weights) for the average.  Returns the reference's shapes: an array, or a
    list / tuple of per-layer arrays (torch tensors on the server GPU when
    the parties held torch tensors)."""
    assert payloads, "Data to aggregate should not be None or empty!"
    p0 = payloads[0]
    names = [p.party for p in payloads]
    assert len(set(names)) == len(names), "each party may contribute one object"
    for p in payloads:
        if (p.sizes, p.shapes, p.container, p.fxp_bits) != (p0.sizes, p0.shapes, p0.container, p0.fxp_bits):
            raise ValueError("parties hold arrays of different shapes")
    fxp_bits = p0.fxp_bits
    n = int(sum(p0.sizes))
    divisor, divisor_vec = 1.0, None
    if average:
        if weights is None:
            divisor = float(len(payloads))
        else:
            weights = [_host_weight(w) for w in weights]
            assert len(weights) == len(payloads), (
                f"Length of the weights does not match the data: {len(weights)} vs {len(payloads)}.")
            if all(np.ndim(w) == 0 for w in weights):
                divisor = float(sum(weights))
            else:
                divisor_vec = [np.concatenate([np.broadcast_to(np.asarray(w), sh).astype(np.float64).reshape(-1)
                                               for sh in p0.shapes]) if n else np.zeros(0)
                               for w in weights]
    dec = _sum_decode_vectors([p.u64 for p in payloads], [p.digest for p in payloads], fxp_bits, divisor,
                              divisor_vec, gpu, p0.as_torch)
    bounds = np.cumsum([0] + list(p0.sizes))
    layers = [dec[int(bounds[i]):int(bounds[i + 1])].reshape(sh) for i, sh in enumerate(p0.shapes)]
    if p0.container == "array":
        return layers[0]
    return tuple(layers) if p0.container == "tuple" else layers


class DigestMismatch(RuntimeError):
    """A masked vector changed between the client and the server."""


def _sum_decode_vectors(u64s, digests, fxp_bits, divisor, divisor_vec, gpu, as_torch):
    """The server's device work: the payloads in (one pinned copy for a small
    call), their XOR digests, the mod-2^64 sum and the decode; the decoded
    result and the digests share one device buffer, so a small host result
    comes back with one copy and one synchronisation."""
    import torch

    from ... import hostpipe as H
    from ... import kernels as K
    from .secure_aggregator import SMALL_CALL_BYTES

    if gpu is None:
        raise RuntimeError("the server has no GPU: libsfl_sa sums on the device")
    dev = torch.device("cuda", gpu)
    n, C = int(u64s[0].size), len(u64s)
    small = 8 * n <= SMALL_CALL_BYTES
    if small and n and not as_torch and divisor_vec is None and C <= 32:
        # ONE blocking library call: the vectors in, digests, sum, decode, the result out
        with _SCRATCH_LOCK, torch.cuda.device(dev):
            pin, dbuf = _scratch(gpu, *K.sum_decode_host_scratch(C, n))
            result, got = K.sum_decode_host(u64s, pin, dbuf, fxp_bits=fxp_bits, divisor=divisor)
        for i, (g, want) in enumerate(zip(got.tolist(), digests)):
            if int(g) != int(want) & ((1 << 64) - 1):
                raise DigestMismatch(f"masked vector {i}: digest {int(g):016x}, sent {int(want):016x}")
        return result
    if not small and not as_torch and divisor_vec is None and LARGE_PIPELINE:
        return _sum_decode_pipelined(u64s, digests, fxp_bits, divisor, dev)
    with torch.cuda.device(dev):
        if small and n:
            n_pad = n + (n & 1)  # rows 16-byte aligned
            pin = torch.empty((C, n_pad), dtype=torch.int64, pin_memory=True)
            pv = pin.numpy()
            for i, u in enumerate(u64s):
                pv[i, :n] = np.asarray(u).view(np.int64)
            dv = pin.to(dev, non_blocking=True)
            vecs = [dv[i, :n] for i in range(C)]
        else:
            vecs = [H.h2d(np.asarray(u).view(np.int64), dev) for u in u64s]
        io = torch.empty(n + C, dtype=torch.float64, device=dev)  # decoded result | digests
        out = io[:n]
        if n:
            dig = io[n:].view(torch.int64)
            dig.zero_()
            for i, v in enumerate(vecs):
                K.xor_digest(v, dig[i:i + 1])
            s = torch.empty(n, dtype=K.U64, device=dev)
            K.sum_u64(vecs, s)
            dv_ = None
            if divisor_vec is not None:
                dv_ = K.sum_f64([H.h2d(w, dev) for w in divisor_vec],
                                torch.empty(n, dtype=torch.float64, device=dev))
            K.decode(s, out, fxp_bits=fxp_bits, divisor=divisor, divisor_vec=dv_)
            if small and not as_torch:
                pin_io = torch.empty(n + C, dtype=torch.float64, pin_memory=True)
                pin_io.copy_(io, non_blocking=True)
                torch.cuda.current_stream(dev).synchronize()
                hv = pin_io.numpy()
                got = hv[n:].view(np.uint64).tolist()
                result = hv[:n].copy()
            else:
                got = K.as_u64(dig).tolist()
                result = out if as_torch else H.d2h(out)
            for i, (g, want) in enumerate(zip(got, digests)):
                if int(g) != int(want) & ((1 << 64) - 1):
                    raise DigestMismatch(f"masked vector {i}: digest {int(g):016x}, sent {int(want):016x}")
            return result
    return out if as_torch else H.d2h(out)


def _sum_decode_pipelined(u64s, digests, fxp_bits, divisor, dev):
    """The server's large host call, chunked through three streams
    (``sfl_amd/hostpipe.py``): chunk j of every masked vector H2D straight
    from the payloads (staged through pinned slots by a feeder thread), then on the
    device the per-vector XOR digests (accumulated over chunks), the
    mod-2^64 sum and the decode of chunk j, then its D2H into the result (a
    recycled registered buffer, or a fresh array reached through a pinned slot)
    -- overlapped with chunk j+1's copies.  Same kernels and result as the
    one-shot path."""
    import torch

    from ... import hostpipe as H
    from ... import kernels as K

    C, n = len(u64s), int(u64s[0].size)
    ph = H.Phases("sum_decode")
    ins = [np.ascontiguousarray(u).reshape(-1).view(np.int64) for u in u64s]
    bounds = H.chunk_bounds(n)
    out = H.FreshOutput(n, np.float64, bounds)
    s_in, s_k, s_out = H.streams(dev)
    # vectors received from parties in this process sit in pooled (registered)
    # results: copied async as they are; anything else (vectors deserialised
    # from another process) is staged by the feeder (or, SERVER_REGISTER,
    # registered lazily as its copies are reached)
    with torch.cuda.device(dev), H.Pinned(ins, register=SERVER_REGISTER) as pin:
        cur = torch.cuda.current_stream(dev)
        vecs = [torch.empty(n, dtype=K.U64, device=dev) for _ in range(C)]
        s = torch.empty(n, dtype=K.U64, device=dev)
        dec = torch.empty(n, dtype=torch.float64, device=dev)
        dig = torch.zeros(C, dtype=K.U64, device=dev)
        ready = torch.cuda.Event()
        ready.record(cur)
        s_in.wait_event(ready)
        s_k.wait_event(ready)

        copies = [[(v[lo:hi], [(h[lo:hi], 0)]) for v, h in zip(vecs, ins)] for lo, hi in bounds]
        feed = H.Issued(s_in, copies, pin) if pin.ok else H.Feeder(s_in, copies)
        try:
            for j, (lo, hi) in enumerate(bounds):
                e_in, e_k = feed.ready(j), torch.cuda.Event()
                with torch.cuda.stream(s_k):
                    s_k.wait_event(e_in)
                    part = [v[lo:hi] for v in vecs]
                    for i, v in enumerate(part):
                        K.xor_digest(v, dig[i:i + 1])
                    K.sum_u64(part, s[lo:hi])
                    K.decode(s[lo:hi], dec[lo:hi], fxp_bits=fxp_bits, divisor=divisor)
                    e_k.record(s_k)
                out.copy_in(j, dec[lo:hi], s_out, e_k)
            got_h = torch.empty(C, dtype=K.U64, pin_memory=True)
            with torch.cuda.stream(s_k):
                got_h.copy_(dig, non_blocking=True)
            ph.mark("pipeline")
        finally:
            feed.join(check=False)  # the feeder is done with the inputs
            out.close()
            s_k.synchronize()
            s_out.synchronize()
            s_in.synchronize()
            cur.wait_stream(s_k)
        feed.join()
        ph.mark("wait")
    ph.note(pinned=pin.ok, **pin.stats, **out.stats)
    ph.done()
    for i, (g, want) in enumerate(zip(got_h.numpy().view(np.uint64).tolist(), digests)):
        if int(g) != int(want) & ((1 << 64) - 1):
            raise DigestMismatch(f"masked vector {i}: digest {int(g):016x}, sent {int(want):016x}")
    return out.array
