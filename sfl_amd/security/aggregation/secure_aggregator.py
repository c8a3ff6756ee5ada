"""SecureAggregator on MI355X: the drop-in for
``secretflow.security.aggregation.SecureAggregator`` (un-vendored,
``secretflow-lite==1.13.0b0``; constructor ``(device, participants,
fxp_bits=18)`` as subclassed at
``sfl/security/aggregation/stateful_fedgen_aggregator.py:23-33`` and used at
``docs/developer/algorithm/secure_aggregation.ipynb`` cell 16).

Protocol (notebook cell 15, semi-honest, no dropout): every party quantizes
``x*w`` to fixed point ``trunc(x*w*2^fxp)`` (int64 viewed as uint64), adds
``m_uv`` for each peer ``v`` whose name sorts after it and subtracts it
otherwise, where ``m_uv = PCG64(seed_uv).integers(int64.min, int64.max)``;
the server sums the masked uint64 vectors mod 2^64 — the masks cancel — and
decodes ``int64(S) / 2^fxp`` as float64, divided by ``sum(w)`` (or C) for the
average.  All per-element work (quantize, mask expansion, mod-2^64 sums,
decode) runs in the hand-written gfx950 kernels of ``libsfl_sa.so``.

Placement: each party is a ``PYU`` bound to a GPU.  When every party sits on
the server's GPU and the payload is float32 with scalar weights, the clients
are simulated by ONE fused launch (``sa_fused_clients``) that expands each
pair stream once and applies it to both clients; otherwise each party masks
on its own GPU (``sa_mask``), the masked vectors move to the server
(``.to(server)``, the wire) and are summed there (``sa_sum_u64``).  Both give
bit-identical sums.

Small host calls (up to ``SMALL_CALL_BYTES`` a party, co-located parties)
are latency-bound, so each is ONE blocking library call
(``sa_fused_clients_host_f32`` for float32, ``sa_clients_host`` for the
other types: host arrays in, decoded result out); a replay after a flagged
raw 0, wire images, per-element weights or more parties than those calls
take go through the general path above.
"""

from __future__ import annotations

from typing import List

import numpy as np
import torch

from ... import hostpipe as H
from ... import kernels as K
from ... import _lib as L
from ...device import PYU, PYUObject, DeviceObject, reveal
from . import party as P
from .aggregator import Aggregator
from .masker import Masker

_NP2T = {np.dtype(np.float32): torch.float32, np.dtype(np.float64): torch.float64,
         np.dtype(np.int64): torch.int64}
_T2NP = {v: k for k, v in _NP2T.items()}
MAX_FUSED_CLIENTS = 8
# per-party bytes up to which a call is latency-bound (tools/config1_bench.py
# at 9 .. 1M elements): host arrays packed into one pinned copy and host
# results collected after one synchronisation; above it the driver's pageable
# copies, which pipeline their staging, are faster than a host memcpy
# into pinned memory
SMALL_CALL_BYTES = 1 << 20


class _Rejected(Exception):
    """A masking launch flagged a raw PCG64 draw of 0 (SA_FLAG_PRG_REJECT)."""


def _layers(payload):
    if isinstance(payload, (list, tuple)):
        return list(payload), True
    return [payload], False


def _np_dtype(a) -> np.dtype:
    if isinstance(a, torch.Tensor):
        return _T2NP.get(a.dtype) or np.dtype(str(a.dtype).replace("torch.", ""))
    return np.asarray(a).dtype


def _shape(a):
    return tuple(a.shape) if isinstance(a, torch.Tensor) else np.shape(a)


def _compute_dtype(ldt: np.dtype, w, fxp_bits: int) -> np.dtype:
    """Result dtype of ``(datum * w) * (1 << fxp)`` under the numpy the
    reference pins, 1.23.5 (``uv.lock:1189-1190``): value-based casting, so a
    scalar weight -- python OR numpy scalar / 0-d array -- does not widen
    the array's dtype when its value fits (``result_type(dtype,
    min_scalar_type(w))``); array weights promote as usual.  numpy 2's NEP 50
    would make a numpy-scalar weight "strong" (float32 data * np.float64(w)
    -> float64); no reference fixture pins either (parity
    unpinned), the pinned version decides.  Python scalars behave alike
    under both rules."""
    probe = np.zeros(1, dtype=ldt)
    if w is not None:
        if isinstance(w, (bool, int, float)) and not isinstance(w, np.generic):  # np.float64 is a float
            probe = probe * w
        else:
            wa = np.asarray(w)
            dt = np.result_type(ldt, wa.dtype if wa.ndim else np.min_scalar_type(wa))
            probe = probe.astype(dt)
    return (probe * (1 << fxp_bits)).dtype


class SecureAggregator(Aggregator):
    """Pairwise-mask secure aggregation with the HIP hot path.

    Args:
        device: the server PYU that receives the masked vectors and decodes.
        participants: the client PYUs (distinct parties).
        fxp_bits: fixed-point fraction bits (reference default 18).
        seeds: optional ``{(party_a, party_b): seed}`` pairwise seeds (both
            orders accepted; a ``(state, inc)`` tuple is an explicit numpy
            PCG64 state); default is a Diffie-Hellman agreement.
        fused: allow the single-launch simulation of co-located clients.
        keep_masked: also materialise every party's masked vector (the wire
            image) and expose the last ones as ``last_masked``; co-located
            parties still take the fused launch, which stores the images.

    ``last_digests``: per launch group of the last aggregation, the XOR
    digest of every party's masked vector (a checksum the tests pin) -- None
    for a group of more co-located parties than one launch holds, whose
    pair-shared schedule forms only the masked sum.
    """

    def __init__(self, device: PYU, participants: List[PYU], fxp_bits: int = 18, *,
                 seeds: dict | None = None, fused: bool = True, keep_masked: bool = False):
        assert participants, "participants should not be empty"
        names = [p.party for p in participants]
        assert len(set(names)) == len(names), f"duplicate participants: {names}"
        self._device = device
        self._participants = list(participants)
        self._fxp_bits = int(fxp_bits)
        self._fused = fused
        self._keep_masked = keep_masked
        self.last_masked = None
        self.last_digests = None
        self._careful = False  # replay mode after a flagged rejection (see _aggregate)
        self._maskers = {n: Masker(n, self._fxp_bits) for n in names}
        if seeds is None:
            keys = {n: m.public_key for n, m in self._maskers.items()}
            for m in self._maskers.values():
                m.agree(keys)
        else:
            for a in names:
                for b in names:
                    if a != b:
                        s = seeds.get((a, b), seeds.get((b, a)))
                        if s is None:
                            raise ValueError(f"missing seed for pair ({a}, {b})")
                        if isinstance(s, tuple):  # an explicit numpy PCG64 (state, inc)
                            self._maskers[a].set_state(b, *s)
                        else:
                            self._maskers[a].set_seed(b, int(s))

    @property
    def device(self) -> PYU:
        return self._device

    @property
    def participants(self) -> List[PYU]:
        return list(self._participants)

    # ------------------------------------------------------------------ API
    def sum(self, data: List[DeviceObject], axis=None) -> DeviceObject:
        return self._aggregate(data, axis, weights=None, average=False)

    def average(self, data: List[DeviceObject], axis=None, weights=None) -> DeviceObject:
        return self._aggregate(data, axis, weights=weights, average=True)

    # ------------------------------------------------------------ internals
    def _aggregate(self, data, axis, weights, average: bool) -> DeviceObject:
        """One aggregation.  The masking kernels only FLAG a raw PCG64 draw
        of 0 (numpy's Generator.integers rejects it and draws again, p =
        2^-64 per draw); when that happens the round is replayed from the
        same stream positions in careful mode, which re-positions the
        affected streams exactly as numpy does (``_fix_rejections``)."""
        snap = {nm: m.snapshot() for nm, m in self._maskers.items()}

        def restore():
            for nm, m in self._maskers.items():
                m.restore(snap[nm])

        try:
            return self._aggregate_once(data, axis, weights, average)
        except _Rejected:
            restore()
        except BaseException:
            # any other failure part-way through a multi-group round: put every
            # stream back where the peers (and numpy) still have it
            restore()
            raise
        self._careful = True
        try:
            return self._aggregate_once(data, axis, weights, average)
        except BaseException:
            restore()
            raise
        finally:
            self._careful = False

    def _aggregate_once(self, data, axis, weights, average: bool) -> DeviceObject:
        assert data, "Data to aggregate should not be None or empty!"
        if axis not in (0, None):
            raise NotImplementedError("SecureAggregator aggregates over parties (axis=0)")
        for d in data:
            assert isinstance(d, PYUObject), f"expect PYUObject, got {type(d)}"
            assert d.device.party in self._maskers, f"{d.device} is not a participant"
        owners = [d.device.party for d in data]
        assert len(set(owners)) == len(owners), "each party may contribute one object"
        assert set(owners) == set(self._maskers), (
            "every participant must contribute (pairwise masks only cancel without dropout, "
            "secure_aggregation.ipynb cell 15)")
        if weights is not None:
            if isinstance(weights, PYUObject):
                raise TypeError("weights must be a per-party list")
            assert len(weights) == len(data), (
                f"Length of the weights does not match the data: {len(weights)} vs {len(data)}.")
            wl = []
            for i, w in enumerate(weights):
                if isinstance(w, PYUObject):
                    assert w.device == data[i].device, "Device of weight does not match the corresponding data device."
                    w = reveal(w)
                if isinstance(w, torch.Tensor):
                    w = w.detach().numpy() if w.device.type == "cpu" else H.d2h(w, pooled=False)
                wl.append(w)
            weights = wl

        payloads = [d.data for d in data]
        layer_lists, is_list = zip(*[_layers(p) for p in payloads])
        is_list = is_list[0]
        nl = len(layer_lists[0])
        for ll in layer_lists:
            assert len(ll) == nl, "parties hold different numbers of arrays"
        shapes = [_shape(a) for a in layer_lists[0]]
        for ll in layer_lists:
            assert [_shape(a) for a in ll] == shapes, "parties hold arrays of different shapes"
        as_torch = isinstance(layer_lists[0][0], torch.Tensor)

        server = self._device
        sdev = server.torch_device
        masked_keep, digests_keep = [], []

        # layers are masked in order with one stream position per (party, peer),
        # exactly like the reference's per-layer rng.integers calls
        sizes = [int(np.prod(sh)) if sh else 1 for sh in shapes]
        if self._host_fusable(data, layer_lists, as_torch, weights, sum(sizes)):
            return self._aggregate_host_fused(data, layer_lists, sizes, shapes, weights, average, is_list,
                                              payloads, digests_keep)
        if not as_torch:
            res = self._host_general_one_call(data, layer_lists, sizes, shapes, weights, average, is_list,
                                              payloads, digests_keep)
            if res is not None:
                return res
        flags = torch.zeros(1, dtype=torch.int32, device=sdev)
        if (nl > 1 and not as_torch and (weights is None or all(np.ndim(w) == 0 for w in weights))
                and all(len({np.asarray(a).dtype for a in ll}) == 1 for ll in layer_lists)):
            # host payloads of one dtype: pack on the host, one H2D copy per party
            flat = [np.concatenate([np.asarray(a).reshape(-1) for a in ll]) for ll in layer_lists]
            g = self._prepare_layer(data, flat, (sum(sizes),), weights)
            return self._finish(data, [(list(range(nl)), sizes, g)], shapes, weights, average, as_torch,
                                is_list, payloads, flags, masked_keep, digests_keep)
        prepared = [self._prepare_layer(data, [ll[li] for ll in layer_lists], shapes[li], weights)
                    for li in range(nl)]
        # Consecutive layers draw consecutive stream positions, so when every
        # layer of a party has the same element/arithmetic type and a scalar
        # weight, the layers are packed into one contiguous vector per party
        # (List[array] <-> one vector + offsets) and aggregated
        # by ONE launch -- bit-identical to the per-layer launches.
        packable = nl > 1 and all(
            all(p["wvecs"][ci] is None and p["xs"][ci].dtype == prepared[0]["xs"][ci].dtype
                and p["cts"][ci] == prepared[0]["cts"][ci] for p in prepared)
            for ci in range(len(data)))
        if packable:
            groups = [(list(range(nl)), sizes, {
                "n": sum(sizes), "cts": prepared[0]["cts"], "ws": prepared[0]["ws"],
                "wvecs": [None] * len(data),
                "xs": [torch.cat([p["xs"][ci] for p in prepared]) for ci in range(len(data))]})]
        else:
            groups = [([li], [prepared[li]["n"]], prepared[li]) for li in range(nl)]

        return self._finish(data, groups, shapes, weights, average, as_torch, is_list, payloads, flags,
                            masked_keep, digests_keep)

    # ------------------------------------------- host payloads, one launch
    def _host_fusable(self, data, layer_lists, as_torch, weights, n) -> bool:
        """Host float32 payloads of co-located parties with scalar weights that
        keep float32 arithmetic: the latency path below applies (FL rounds
        of small models)."""
        if as_torch or not self._fused or self._keep_masked or n == 0:
            return False
        if len(data) < 2 or (len(data) > MAX_FUSED_CLIENTS and self._careful):
            return False
        sgpu = self._device.gpu
        if any(d.device.gpu != sgpu for d in data):
            return False
        f32 = np.dtype(np.float32)
        for i, ll in enumerate(layer_lists):
            if any(_np_dtype(a) != f32 for a in ll):
                return False
            w = None if weights is None else weights[i]
            if w is not None and (np.ndim(w) != 0 or _compute_dtype(f32, w, self._fxp_bits) != f32):
                return False
        return True

    def _staging(self, C: int, n_pad: int, sdev):
        """Pinned host / device buffers reused across rounds of the same size:
        the input block [C, n_pad] float32 (host and device), the masked-sum
        buffer, and one float64 block ``io`` of n_pad + 1 + C words on the
        device with its pinned host mirror -- the decoded result, then a word
        whose low half is the PRG flag word, then the C digests -- so that ONE
        zero fill and ONE device-to-host copy serve all three."""
        key = (C, n_pad, str(sdev))
        st = getattr(self, "_stage", None)
        if st is None or st["key"] != key:
            io_dev = torch.empty(n_pad + 1 + C, dtype=torch.float64, device=sdev)
            io_host = torch.empty(n_pad + 1 + C, dtype=torch.float64, pin_memory=True)
            meta = io_dev[n_pad:].view(torch.int64)
            small = 4 * n_pad <= SMALL_CALL_BYTES  # large calls copy from the caller's arrays
            st = {"key": key,
                  "in_host": torch.empty((C, n_pad) if small else (0, 0), dtype=torch.float32, pin_memory=True),
                  "in_dev": torch.empty((C, n_pad), dtype=torch.float32, device=sdev),
                  "sum": torch.empty(n_pad, dtype=K.U64, device=sdev),
                  "io_dev": io_dev, "io_host": io_host, "meta": meta,
                  "flags": meta[:1].view(torch.int32)[:1], "digests": meta[1:],
                  "io_f64": io_host.numpy(), "io_i64": io_host.numpy().view(np.int64)}
            st["in_np"] = st["in_host"].numpy()
            self._stage = st
        return st

    def _aggregate_host_fused(self, data, layer_lists, sizes, shapes, weights, average, is_list, payloads,
                              digests_keep):
        """Small calls (up to SMALL_CALL_BYTES a party): ONE blocking library
        call (``_host_one_call``: the parties' layers packed into one pinned
        block, one H2D copy, one zero fill of the PRG flag + digests, the
        fused masking launch -- same kernels and stream positions as the
        general path: bit-identical -- decode, one D2H copy of the result
        with the flag word and the digests, one synchronisation); the same
        steps from Python when a replay (careful mode) or more than 8 parties
        need the general machinery.  Large calls copy each party's array and
        the result directly."""
        sdev = self._device.torch_device
        C, n = len(data), sum(sizes)
        n_pad = -(-n // 4) * 4  # rows start 16-byte aligned
        # small calls: one pinned block, one copy; large ones: the driver's
        # pageable copy per party (its staging pipelines, a host memcpy into
        # pinned memory first does not)
        big = 4 * n_pad > SMALL_CALL_BYTES
        if big and not self._careful and P.LARGE_PIPELINE:
            return self._host_fused_pipelined(data, layer_lists, sizes, shapes, weights, average, is_list,
                                              payloads, digests_keep, C, n, sdev)
        if not big and not self._careful and C <= MAX_FUSED_CLIENTS:
            res = self._host_one_call(data, layer_lists, sizes, shapes, weights, average, is_list, payloads,
                                      digests_keep, C, n, sdev)
            if res is not None:
                return res
        st = self._staging(C, n_pad, sdev)
        host = st["in_np"]
        with torch.cuda.device(sdev):
            dev_in = st["in_dev"]
            for c, ll in enumerate(layer_lists):
                if big:
                    src = (np.asarray(ll[0], dtype=np.float32).reshape(-1) if len(ll) == 1 else
                           np.concatenate([np.asarray(a, dtype=np.float32).reshape(-1) for a in ll]))
                    dev_in[c, :n].copy_(H.h2d(src, sdev))
                elif len(ll) == 1:
                    host[c, :n] = np.asarray(ll[0], dtype=np.float32).reshape(-1)
                else:
                    np.concatenate([np.asarray(a, dtype=np.float32).reshape(-1) for a in ll], out=host[c, :n])
            if not big:
                dev_in.copy_(st["in_host"], non_blocking=True)
            st["meta"].zero_()
            xs = [dev_in[c, :n] for c in range(C)]
            ws = [1.0 if weights is None else float(w) for w in (weights or [None] * C)]
            s = self._masked_sum(data, xs, [np.dtype(np.float32)] * C, ws, [None] * C, n, st["flags"], [],
                                 digests_keep, s_out=st["sum"][:n], digests_out=st["digests"])
            divisor = 1.0
            if average:
                divisor = float(C) if weights is None else float(sum(weights))
            K.decode(s, st["io_dev"][:n], fxp_bits=self._fxp_bits, divisor=divisor)
            if big:
                out = H.d2h(st["io_dev"][:n])
                st["io_host"][n_pad:].copy_(st["io_dev"][n_pad:])
            else:
                st["io_host"].copy_(st["io_dev"], non_blocking=True)
                torch.cuda.current_stream(sdev).synchronize()
        io64, ioi = st["io_f64"], st["io_i64"]
        if not big:
            out = io64[:n].copy()
        if int(ioi[n_pad]) & L.SA_FLAG_PRG_REJECT:  # the flag word's low half (little-endian)
            raise _Rejected()
        self.last_digests = [None if d is None else torch.from_numpy(ioi[n_pad + 1:n_pad + 1 + C].copy())
                             for d in digests_keep]
        parts = np.split(out, np.cumsum(sizes)[:-1]) if len(sizes) > 1 else [out]
        result = [p.reshape(sh) for p, sh in zip(parts, shapes)]
        if not is_list:
            return PYUObject(self._device, result[0])
        return PYUObject(self._device, tuple(result) if isinstance(payloads[0], tuple) else result)

    def _host_fused_pipelined(self, data, layer_lists, sizes, shapes, weights, average, is_list, payloads,
                              digests_keep, C, n, sdev):
        """Large host float32 payloads of co-located parties, chunked
        through three streams (``sfl_amd/hostpipe.py``, as the per-party
        drop-in's large path): chunk j of every party's layers H2D straight
        from the caller's arrays (registered for the call, else staged
        through pinned slots by a feeder thread), the fused launch of chunk j
        (every pair stream advanced to ``lo``, digests and the PRG flag
        accumulated on the device) and its decode, then the D2H of chunk j
        into the result (a recycled registered buffer, or a fresh array
        reached through a pinned slot).  Bit-identical to one fused launch over
        [0, n); more than 8 parties take the pair-shared schedule per chunk
        (``kernels.fused_many``: the sum only, no per-party digests)."""
        from ... import hostpipe as H

        ph = H.Phases("average" if average else "sum")
        names = [d.device.party for d in data]
        pair_gens, pair_signs = self._pair_streams(names)
        ws = [1.0 if weights is None else float(w) for w in (weights or [None] * C)]
        divisor = 1.0
        if average:
            divisor = float(C) if weights is None else float(sum(weights))
        layers = [H.host_layers(ll, np.float32) for ll in layer_lists]
        n_pad = -(-n // 4) * 4  # rows 16-byte aligned
        bounds = H.page_bounds(H.chunk_bounds(n), layers)
        out = H.FreshOutput(n, np.float64, bounds)  # its pages start faulting in now
        s_in, s_k, s_out = H.streams(sdev)
        with torch.cuda.device(sdev), H.Pinned([a for ls in layers for a in ls]) as pin:
            ph.mark("register in")
            cur = torch.cuda.current_stream(sdev)
            x = torch.empty((C, n_pad), dtype=torch.float32, device=sdev)
            ssum = torch.empty(n, dtype=K.U64, device=sdev)
            dec = torch.empty(n, dtype=torch.float64, device=sdev)
            meta = torch.zeros(1 + C, dtype=K.U64, device=sdev)  # flag word | digests
            # more parties than one launch holds: the pair-shared schedule
            # (kernels.fused_many) forms only the sum, no per-party digests
            flags, digests = meta[:1].view(torch.int32)[:1], (meta[1:] if C <= MAX_FUSED_CLIENTS else None)
            ready = torch.cuda.Event()
            ready.record(cur)
            s_in.wait_event(ready)
            s_k.wait_event(ready)

            copies = [[(x[c, lo:hi], H.pieces(layers[c], lo, hi)) for c in range(C)] for lo, hi in bounds]
            # registered layers: every H2D issued at once, async; else staged by the feeder
            feed = H.Issued(s_in, copies, pin) if pin.ok else H.Feeder(s_in, copies)
            try:
                for j, (lo, hi) in enumerate(bounds):
                    gens = L.pcg64_advance_many(pair_gens, [lo] * len(pair_gens)) if lo else pair_gens
                    e_in, e_k = feed.ready(j), torch.cuda.Event()
                    with torch.cuda.stream(s_k):
                        s_k.wait_event(e_in)
                        K.fused_clients([x[c, lo:hi] for c in range(C)], ws, gens, pair_signs, [], 0, ssum[lo:hi],
                                        fxp_bits=self._fxp_bits, digests=digests, flags=flags)
                        K.decode(ssum[lo:hi], dec[lo:hi], fxp_bits=self._fxp_bits, divisor=divisor)
                        e_k.record(s_k)
                    out.copy_in(j, dec[lo:hi], s_out, e_k)
                meta_h = torch.empty(1 + C, dtype=K.U64, pin_memory=True)
                with torch.cuda.stream(s_k):
                    meta_h.copy_(meta, non_blocking=True)
                ph.mark("pipeline")
            finally:
                feed.join(check=False)  # the feeder is done with the inputs
                out.close()
                s_k.synchronize()
                s_out.synchronize()
                s_in.synchronize()
                cur.wait_stream(s_k)  # x, ssum, dec, meta were allocated on the current stream
            feed.join()
            ph.mark("wait")
        ph.mark("unregister")
        ph.note(pinned=pin.ok, **pin.stats, **out.stats)
        ph.done()
        mh = meta_h.numpy()
        if int(mh[0]) & L.SA_FLAG_PRG_REJECT:  # the flag word's low half (little-endian)
            raise _Rejected()
        for nm in names:
            self._maskers[nm].consume(n)
        digests_keep.append(torch.from_numpy(mh[1:].copy()) if C <= MAX_FUSED_CLIENTS else None)
        self.last_digests = digests_keep
        res = out.array
        parts = np.split(res, np.cumsum(sizes)[:-1]) if len(sizes) > 1 else [res]
        result = [p.reshape(sh) for p, sh in zip(parts, shapes)]
        if not is_list:
            return PYUObject(self._device, result[0])
        return PYUObject(self._device, tuple(result) if isinstance(payloads[0], tuple) else result)

    def _pair_streams(self, names, want: bool = True):
        """Every internal pair (u < v) of ``names``: its generator at the next
        unused draw (u's view, one library call per party) and u's sign,
        u-major -- the order sa_fused_clients takes."""
        C = len(names)
        gens, signs = [], []
        for u in range(C):
            mu = self._maskers[names[u]]
            later = names[u + 1:]
            for v in later:
                assert mu.position(v) == self._maskers[v].position(names[u]), "pair streams out of step"
            if want and later:
                gens += mu.generators_at(later)
                signs += [mu.sign(v) for v in later]
        return gens, signs

    def _host_one_call(self, data, layer_lists, sizes, shapes, weights, average, is_list, payloads, digests_keep,
                       C, n, sdev):
        """The small call as ONE blocking library call
        (``sa_fused_clients_host_f32``: host arrays in, decoded result,
        digests and PRG flag out; the Python side only positions the pair
        streams).  None when the library has no fused kernel for C."""
        names = [d.device.party for d in data]
        pair_gens, pair_signs = self._pair_streams(names)
        key = (C, n, str(sdev))
        sc = getattr(self, "_one_call", None)
        if sc is None or sc[0] != key:
            pin_b, dev_b = K.host_fused_scratch(C, n)
            sc = (key, torch.empty(pin_b, dtype=torch.uint8, pin_memory=True),
                  torch.empty(dev_b, dtype=torch.uint8, device=sdev))
            self._one_call = sc
        xs = [ll[0] if len(ll) == 1 else np.concatenate([np.asarray(a, dtype=np.float32).reshape(-1) for a in ll])
              for ll in layer_lists]
        ws = [1.0 if weights is None else float(w) for w in (weights or [None] * C)]
        divisor = 1.0
        if average:
            divisor = float(C) if weights is None else float(sum(weights))
        with torch.cuda.device(sdev):
            got = K.fused_clients_host_f32(xs, ws, pair_gens, pair_signs, sc[1], sc[2], fxp_bits=self._fxp_bits,
                                           divisor=divisor)
        if got is None:
            return None
        out, digests, flag = got
        if flag & L.SA_FLAG_PRG_REJECT:
            raise _Rejected()
        for nm in names:
            self._maskers[nm].consume(n)
        digests_keep.append(torch.from_numpy(digests.view(np.int64)))
        self.last_digests = digests_keep
        parts = np.split(out, np.cumsum(sizes)[:-1]) if len(sizes) > 1 else [out]
        result = [p.reshape(sh) for p, sh in zip(parts, shapes)]
        if not is_list:
            return PYUObject(self._device, result[0])
        return PYUObject(self._device, tuple(result) if isinstance(payloads[0], tuple) else result)

    def _host_general_shape(self, data, layer_lists, weights, n):
        """(element type, compute type, scalar weights) of host payloads of
        one element type in ``_NP2T`` with scalar weights of one compute type,
        every party on the server's GPU -- the shape the general host paths
        below take -- else None."""
        C = len(data)
        if (self._careful or self._keep_masked or not self._fused or C < 2 or n == 0
                or any(d.device.gpu != self._device.gpu for d in data)):
            return None
        if weights is not None and any(np.ndim(w) for w in weights):
            return None
        try:
            dts = {np.asarray(a).dtype for ll in layer_lists for a in ll}
        except Exception:  # noqa: BLE001 - ragged or exotic payloads: the general path decides
            return None
        if len(dts) != 1:
            return None
        xt = dts.pop()
        if xt not in _NP2T:
            return None
        cts = {_compute_dtype(xt, None if weights is None else weights[i], self._fxp_bits) for i in range(C)}
        if len(cts) != 1:
            return None
        ct = cts.pop()
        if ct not in _NP2T:
            return None
        ws = [1.0 if weights is None else (float(w) if ct.kind == "f" else int(w)) for w in (weights or [None] * C)]
        return xt, ct, ws

    def _host_general_one_call(self, data, layer_lists, sizes, shapes, weights, average, is_list, payloads,
                               digests_keep):
        """Host calls of float64 / int64 data (or float32 data with a float64
        compute type) of 2..9 parties on the server's GPU: small ones as ONE
        blocking library call (``sa_clients_host``: every party masked with
        its own streams into the sum, decode, one copy each way), large ones
        (any number of parties) chunked through ``_host_general_pipelined``.
        None when the call is of neither shape (the general path takes it)."""
        C, n = len(data), sum(sizes)
        got = self._host_general_shape(data, layer_lists, weights, n)
        if got is None:
            return None
        xt, ct, ws = got
        if n * xt.itemsize > SMALL_CALL_BYTES:
            if not P.LARGE_PIPELINE:
                return None
            return self._host_general_pipelined(data, layer_lists, sizes, shapes, weights, average, is_list,
                                                payloads, digests_keep, xt, ct, ws)
        if C > 9:
            return None
        names = [d.device.party for d in data]
        streams = [self._maskers[nm].streams(self._maskers[nm].peers) for nm in names]
        xs = [np.asarray(ll[0]).reshape(-1) if len(ll) == 1 else
              np.concatenate([np.asarray(a).reshape(-1) for a in ll]) for ll in layer_lists]
        sdev = self._device.torch_device
        key = (C, n, xt.itemsize, str(sdev))
        sc = getattr(self, "_general_call", None)
        if sc is None or sc[0] != key:
            pin_b, dev_b = K.host_clients_scratch(C, n, xt.itemsize)
            sc = (key, torch.empty(pin_b, dtype=torch.uint8, pin_memory=True),
                  torch.empty(dev_b, dtype=torch.uint8, device=sdev))
            self._general_call = sc
        divisor = 1.0
        if average:
            divisor = float(C) if weights is None else float(sum(weights))
        with torch.cuda.device(sdev):
            out, digests, flag = K.clients_host(xs, ct, ws, streams, sc[1], sc[2], fxp_bits=self._fxp_bits,
                                                divisor=divisor)
        if flag & L.SA_FLAG_PRG_REJECT:
            raise _Rejected()
        for nm in names:
            self._maskers[nm].consume(n)
        digests_keep.append(torch.from_numpy(digests.view(np.int64)))
        self.last_digests = digests_keep
        parts = np.split(out, np.cumsum(sizes)[:-1]) if len(sizes) > 1 else [out]
        result = [p.reshape(sh) for p, sh in zip(parts, shapes)]
        if not is_list:
            return PYUObject(self._device, result[0])
        return PYUObject(self._device, tuple(result) if isinstance(payloads[0], tuple) else result)

    def _host_general_pipelined(self, data, layer_lists, sizes, shapes, weights, average, is_list, payloads,
                                digests_keep, xt, ct, ws):
        """Large host payloads of the general shape (``_host_general_shape``:
        float64 / int64 data, or float32 data computed in float64), chunked
        through the three streams exactly like ``_host_fused_pipelined``:
        chunk j of every party H2D (registered inputs issued async, else
        staged by the feeder), then on the compute stream every party's
        ``sa_mask`` of chunk j with its own streams advanced to ``lo``
        accumulating into the sum (its digest and the PRG flag accumulated on
        the device), the decode of chunk j, and its D2H into the result.
        Bit-identical to the one-shot general path: the same kernel, the same
        stream positions, element by element."""
        from ... import hostpipe as H

        sdev = self._device.torch_device
        C, n = len(data), sum(sizes)
        ph = H.Phases("average" if average else "sum")
        names = [d.device.party for d in data]
        divisor = 1.0
        if average:
            divisor = float(C) if weights is None else float(sum(weights))
        tx, tc = _NP2T[xt], _NP2T[ct]
        layers = [H.host_layers(ll, xt) for ll in layer_lists]
        n_pad = -(-n // 4) * 4  # rows 16-byte aligned
        bounds = H.page_bounds(H.chunk_bounds(n), layers)
        out = H.FreshOutput(n, np.float64, bounds)
        s_in, s_k, s_out = H.streams(sdev)
        with torch.cuda.device(sdev), H.Pinned([a for ls in layers for a in ls]) as pin:
            ph.mark("register in")
            cur = torch.cuda.current_stream(sdev)
            x = torch.empty((C, n_pad), dtype=tx, device=sdev)
            ssum = torch.empty(n, dtype=K.U64, device=sdev)
            dec = torch.empty(n, dtype=torch.float64, device=sdev)
            masked = torch.empty(max(hi - lo for lo, hi in bounds), dtype=K.U64, device=sdev)
            meta = torch.zeros(1 + C, dtype=K.U64, device=sdev)  # flag word | digests
            flags = meta[:1].view(torch.int32)[:1]
            ready = torch.cuda.Event()
            ready.record(cur)
            s_in.wait_event(ready)
            s_k.wait_event(ready)

            copies = [[(x[c, lo:hi], H.pieces(layers[c], lo, hi)) for c in range(C)] for lo, hi in bounds]
            feed = H.Issued(s_in, copies, pin) if pin.ok else H.Feeder(s_in, copies)
            try:
                for j, (lo, hi) in enumerate(bounds):
                    streams = [self._maskers[nm].streams(offset=lo) for nm in names]
                    e_in, e_k = feed.ready(j), torch.cuda.Event()
                    with torch.cuda.stream(s_k):
                        s_k.wait_event(e_in)
                        ssum[lo:hi].zero_()
                        for c in range(C):
                            K.mask(x[c, lo:hi], masked[:hi - lo], streams[c], weight=ws[c], compute_dtype=tc,
                                   fxp_bits=self._fxp_bits, sum_accum=ssum[lo:hi], digest=meta[1 + c:2 + c],
                                   flags=flags)
                        K.decode(ssum[lo:hi], dec[lo:hi], fxp_bits=self._fxp_bits, divisor=divisor)
                        e_k.record(s_k)
                    out.copy_in(j, dec[lo:hi], s_out, e_k)
                meta_h = torch.empty(1 + C, dtype=K.U64, pin_memory=True)
                with torch.cuda.stream(s_k):
                    meta_h.copy_(meta, non_blocking=True)
                ph.mark("pipeline")
            finally:
                feed.join(check=False)
                out.close()
                s_k.synchronize()
                s_out.synchronize()
                s_in.synchronize()
                cur.wait_stream(s_k)  # x, ssum, dec, masked, meta were allocated on the current stream
            feed.join()
            ph.mark("wait")
        ph.mark("unregister")
        ph.note(pinned=pin.ok, **pin.stats, **out.stats)
        ph.done()
        mh = meta_h.numpy()
        if int(mh[0]) & L.SA_FLAG_PRG_REJECT:  # the flag word's low half (little-endian)
            raise _Rejected()
        for nm in names:
            self._maskers[nm].consume(n)
        digests_keep.append(torch.from_numpy(mh[1:].copy()))
        self.last_digests = digests_keep
        res = out.array
        parts = np.split(res, np.cumsum(sizes)[:-1]) if len(sizes) > 1 else [res]
        result = [p.reshape(sh) for p, sh in zip(parts, shapes)]
        if not is_list:
            return PYUObject(self._device, result[0])
        return PYUObject(self._device, tuple(result) if isinstance(payloads[0], tuple) else result)

    def _finish(self, data, groups, shapes, weights, average, as_torch, is_list, payloads, flags, masked_keep,
                digests_keep):
        """Masked sum + decode of every launch group, split back into layers."""
        sdev = self._device.torch_device
        server = self._device
        nl = len(shapes)
        out_layers = [None] * nl
        host_groups = []
        for lis, sizes, g in groups:
            n = g["n"]
            keep_before = len(masked_keep)
            s = self._masked_sum(data, g["xs"], g["cts"], g["ws"], g["wvecs"], n, flags, masked_keep,
                                 digests_keep)
            if self._keep_masked and len(lis) > 1:
                packed = masked_keep.pop(keep_before)
                bounds = np.cumsum([0] + sizes)
                for k in range(len(lis)):
                    masked_keep.append([m[bounds[k]:bounds[k + 1]] for m in packed])

            # decode on the server GPU: / 2^fxp, then / C or / sum(w)
            dec = torch.empty(n, dtype=torch.float64, device=sdev)
            divisor, divisor_vec = 1.0, None
            if average:
                if weights is None:
                    divisor = float(len(data))
                elif all(np.ndim(w) == 0 for w in weights):
                    divisor = float(sum(weights))
                else:
                    li = lis[0]
                    wb = [H.h2d(np.broadcast_to(np.asarray(w), shapes[li]).astype(np.float64).reshape(-1), sdev)
                          for w in weights]
                    divisor_vec = K.sum_f64(wb, torch.empty(n, dtype=torch.float64, device=sdev))
            K.decode(s, dec, fxp_bits=self._fxp_bits, divisor=divisor, divisor_vec=divisor_vec)
            if as_torch:
                for li, part in zip(lis, dec.split(sizes)):
                    out_layers[li] = part.reshape(shapes[li])
            elif 8 * n > SMALL_CALL_BYTES:
                vals = H.d2h(dec)
                for li, part in zip(lis, np.split(vals, np.cumsum(sizes)[:-1])):
                    out_layers[li] = part.reshape(shapes[li])
            else:  # small host results: pinned copies, collected after ONE synchronisation below
                host = torch.empty(n, dtype=torch.float64, pin_memory=True)
                host.copy_(dec, non_blocking=True)
                host_groups.append((lis, sizes, host))

        if not host_groups:
            rejected = int(flags.item()) & L.SA_FLAG_PRG_REJECT
        else:
            fl_host = torch.empty(1, dtype=torch.int32, pin_memory=True)
            fl_host.copy_(flags, non_blocking=True)
            torch.cuda.current_stream(sdev).synchronize()
            rejected = int(fl_host[0]) & L.SA_FLAG_PRG_REJECT
            for lis, sizes, host in host_groups:
                vals = host.numpy().copy()
                for li, part in zip(lis, np.split(vals, np.cumsum(sizes)[:-1]) if len(lis) > 1 else [vals]):
                    out_layers[li] = part.reshape(shapes[li])
        if rejected:
            raise _Rejected()
        if self._keep_masked:
            self.last_masked = masked_keep
        self.last_digests = digests_keep
        result = out_layers if is_list else out_layers[0]
        if is_list and isinstance(payloads[0], tuple):
            result = tuple(result)
        return PYUObject(server, result)

    def _prepare_layer(self, data, arrays, shape, weights) -> dict:
        """Per-party device vector, arithmetic type and weight of one layer."""
        n = int(np.prod(shape)) if shape else 1
        xs, cts, ws, wvecs = [], [], [], []
        packed = self._pack_host(data, arrays, n)
        for ci, d in enumerate(data):
            party = d.device
            a = arrays[ci]
            w = None if weights is None else weights[ci]
            ldt = _np_dtype(a)
            ct = _compute_dtype(ldt, w, self._fxp_bits)
            if ct not in (np.dtype(np.float32), np.dtype(np.float64), np.dtype(np.int64)):
                raise NotImplementedError(f"arithmetic type {ct} (data {ldt}) is not supported")
            xt = ldt if ldt in _NP2T else (np.dtype(np.int64) if ldt.kind in "biu" else np.dtype(np.float64))
            if ldt.kind in "biu" and ldt != np.dtype(np.int64) and ct.kind == "i":
                raise NotImplementedError(f"integer data of type {ldt} is not supported")
            x = packed[ci] if packed.get(ci) is not None and packed[ci].dtype == _NP2T[xt] else \
                self._to_device(a, xt, party)
            wv, wscalar = None, 1.0
            if w is not None:
                if np.ndim(w) == 0:
                    wscalar = float(w) if ct.kind == "f" else int(w)
                else:
                    wb = np.broadcast_to(np.asarray(w), shape).astype(ct)
                    wv = H.h2d(wb.reshape(-1), party.torch_device)
            xs.append(x)
            cts.append(ct)
            ws.append(wscalar)
            wvecs.append(wv)
        return {"n": n, "xs": xs, "cts": cts, "ws": ws, "wvecs": wvecs}

    @staticmethod
    def _pack_host(data, arrays, n) -> dict:
        """Host (numpy) arrays of parties on one GPU with one element type:
        packed into one pinned block, ONE host-to-device copy per GPU (the
        small calls of secondary callers, e.g. HomoBinning's counts, are
        bound by per-copy latency).  Returns {party index: device row}."""
        groups = {}
        for ci, d in enumerate(data):
            a = arrays[ci]
            if isinstance(a, torch.Tensor) or n == 0:
                continue
            a = np.asarray(a)
            if a.dtype not in _NP2T or n * a.dtype.itemsize > SMALL_CALL_BYTES:
                continue
            groups.setdefault((d.device.torch_device, a.dtype), []).append(ci)
        rows = {}
        for (dev, dt), cis in groups.items():
            if len(cis) < 2:
                continue
            per = 16 // dt.itemsize
            n_pad = -(-n // per) * per  # every row 16-byte aligned
            host = torch.empty((len(cis), n_pad), dtype=_NP2T[dt], pin_memory=True)
            hv = host.numpy()
            for r, ci in enumerate(cis):
                hv[r, :n] = np.asarray(arrays[ci]).reshape(-1)
            dv = host.to(dev, non_blocking=True)
            for r, ci in enumerate(cis):
                rows[ci] = dv[r, :n]
        return rows

    @staticmethod
    def _to_device(a, xt: np.dtype, party: PYU) -> torch.Tensor:
        tdt = _NP2T[xt]
        if isinstance(a, torch.Tensor) and a.device.type != "cpu":
            t = a.detach().reshape(-1).to(device=party.torch_device, dtype=tdt)
        elif isinstance(a, torch.Tensor):  # cast on the host (no DMA), then a pinned copy
            t = H.h2d(a.detach().reshape(-1).to(tdt), party.torch_device)
        else:
            t = H.h2d(np.ascontiguousarray(np.asarray(a), dtype=xt).reshape(-1), party.torch_device)
        t = t.contiguous()
        if t.data_ptr() % 16:
            t = t.clone()
        return t

    def _masked_sum(self, data, xs, cts, ws, wvecs, n, flags, masked_keep, digests_keep, *, s_out=None,
                    digests_out=None):
        """``s_out`` / ``digests_out``: preallocated sum (n) and zeroed digest
        (C) buffers on the server GPU (the host latency path's staging)."""
        server = self._device
        sdev = server.torch_device
        parties = [d.device for d in data]
        names = [p.party for p in parties]
        C = len(names)
        s = torch.empty(n, dtype=K.U64, device=sdev) if s_out is None else s_out
        # more co-located parties than one launch holds: the pair-shared
        # multi-launch schedule (kernels.fused_many), which forms only the sum
        # (no per-party digests; wire images and the careful replay take the
        # per-party path below)
        many = C > MAX_FUSED_CLIENTS
        if many:
            digests = None
        else:
            digests = torch.zeros(C, dtype=K.U64, device=sdev) if digests_out is None else digests_out
        fusable = (self._fused and C >= 2 and (not many or not (self._keep_masked or self._careful))
                   and all(p.gpu == server.gpu for p in parties)
                   and all(ct == np.dtype(np.float32) for ct in cts)
                   and all(x.dtype == torch.float32 for x in xs)
                   and all(wv is None for wv in wvecs)
                   and set(names) == set(self._maskers))
        # the pair streams (one host jump-ahead each) only where a path uses
        # them: the fused launch and the careful replay's rejection search
        want_pairs = fusable or self._careful
        pair_gens, pair_signs = self._pair_streams(names, want_pairs)
        # per-party (generator, sign, peer) lists: the wire path's launches and the
        # careful-mode rejection fix-up need them (built lazily: 7 jump-aheads a party)
        client_streams = (None if fusable and not self._careful else
                          [self._maskers[p.party].streams(self._maskers[p.party].peers) for p in parties])
        if fusable:
            # keep_masked: the same launch also stores every party's masked
            # vector (the wire image) -- pair streams are still expanded once
            masked = [torch.empty(n, dtype=K.U64, device=sdev) for _ in range(C)] if self._keep_masked else None
            with torch.cuda.device(sdev):
                K.fused_clients(xs, ws, pair_gens, pair_signs, [], 0, s, fxp_bits=self._fxp_bits,
                                digests=digests, flags=flags, masked_outs=masked)
            if self._keep_masked:
                masked_keep.append(masked)
        else:
            if digests is None:
                digests = torch.zeros(C, dtype=K.U64, device=sdev) if digests_out is None else digests_out
            masked = []
            for ci, p in enumerate(parties):
                pdev = p.torch_device
                local = pdev == sdev
                out = torch.empty(n, dtype=K.U64, device=pdev)
                # a party on the server's GPU writes its digest and flag in place
                dig = digests[ci:ci + 1] if local else torch.zeros(1, dtype=K.U64, device=pdev)
                fl = flags if local else torch.zeros(1, dtype=torch.int32, device=pdev)
                with torch.cuda.device(pdev):
                    K.mask(xs[ci], out, client_streams[ci], weight=ws[ci], weight_vec=wvecs[ci],
                           compute_dtype=_NP2T[cts[ci]], fxp_bits=self._fxp_bits, digest=dig, flags=fl)
                if not local:
                    flags |= fl.to(sdev)
                    digests[ci] = dig.to(sdev)[0]
                masked.append(out if local else out.to(sdev))   # the wire: masked vector to the server
            with torch.cuda.device(sdev):
                K.sum_u64(masked, s)
            if self._keep_masked:
                masked_keep.append(masked)
        wire = masked  # materialised masked vectors (None: fused launch without wire images)
        extra = {}
        if self._careful:
            torch.cuda.synchronize(sdev)
            if int(flags.item()) & L.SA_FLAG_PRG_REJECT:
                extra = self._fix_rejections(names, pair_gens, pair_signs, client_streams, xs, ws, wvecs, cts, n,
                                             wire, digests, s)
                flags.zero_()
        for ci, p in enumerate(parties):
            self._maskers[p.party].consume(n)
        for (a, b), k in extra.items():  # the rejected raw draws consumed on top
            self._maskers[a].skip(b, k)
            self._maskers[b].skip(a, k)
        digests_keep.append(digests)
        return s

    def _fix_rejections(self, names, pair_gens, pair_signs, client_streams, xs, ws, wvecs, cts, n, wire, digests,
                        s) -> dict:
        """numpy's rejection re-draw for one launch group (careful mode).

        For every pair stream: the elements from which it runs one more raw
        draw along (``kernels.rejected_draws``); the two clients' masked
        vectors are shifted there (``sa_stream_shift``, opposite signs, so
        the masked sum is unchanged) and their digests recomputed.  Without
        materialised vectors (fused launch, no wire images) an affected
        client's vector is re-masked into scratch for its digest.  Returns
        {(party_a, party_b): extra raw draws} for the stream positions."""
        sdev = self._device.torch_device
        C = len(names)
        fixes = {c: [] for c in range(C)}  # client -> [(gen, sign, points)]
        extra = {}
        # one batched search over every pair stream first (64 generators per
        # launch); only streams with a hit are followed further
        found = K.rejected_draws_many(pair_gens, n, sdev)
        p = 0
        for u in range(C):
            for v in range(u + 1, C):
                pts, total = found[p]
                if pts:
                    fixes[u].append((pair_gens[p], pair_signs[p], pts))
                    fixes[v].append((pair_gens[p], -pair_signs[p], pts))
                    extra[(names[u], names[v])] = total - n
                p += 1
        for c in range(C):
            if not fixes[c]:
                continue
            if wire is not None:
                vec = wire[c]
            else:
                vec = torch.empty(n, dtype=K.U64, device=sdev)
                K.mask(xs[c], vec, client_streams[c], weight=ws[c], weight_vec=wvecs[c],
                       compute_dtype=_NP2T[cts[c]], fxp_bits=self._fxp_bits)
            for gen, sign, pts in fixes[c]:
                for k, shift in pts:
                    K.stream_shift(vec, gen, sign, k, shift)
            digests[c] = 0
            K.xor_digest(vec, digests[c:c + 1])
        if wire is not None:  # the server sums the wire images it received
            K.sum_u64(wire, s)
        return extra
