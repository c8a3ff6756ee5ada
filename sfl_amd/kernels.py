"""Tensor-level wrappers of the HIP hot path (libsfl_sa.so via ctypes).

PyTorch is plumbing here: it owns device memory and streams; the work is done
by the hand-written gfx950 kernels behind the C-ABI.  uint64 buffers are
carried as ``torch.int64`` tensors (same bits); ``as_u64`` gives numpy views.

Every function launches asynchronously on the current torch stream of the
tensors' device and raises ``SALibraryError`` on any error.  Nothing here
falls back to a CPU implementation.
"""

from __future__ import annotations

import ctypes as C
from typing import Sequence

import numpy as np
import torch

from . import _lib as L

U64 = torch.int64  # storage dtype for uint64 buffers

_XTYPE = {torch.float32: L.SA_F32, torch.float64: L.SA_F64, torch.int64: L.SA_I64}


_raw_stream = getattr(torch._C, "_cuda_getCurrentRawStream", None)


def _stream(t: torch.Tensor) -> int:
    """The current torch stream of ``t``'s device, as the raw handle the C-ABI
    takes (torch's raw-stream binding costs ~1 us where
    ``torch.cuda.current_stream(device)`` costs ~5 us: small calls launch
    several kernels, tools/latency_profile.py)."""
    if _raw_stream is not None:
        return _raw_stream(t.device.index)
    return torch.cuda.current_stream(t.device).cuda_stream


def _ptr(t):
    return None if t is None else C.c_void_p(t.data_ptr())


def _require_gpu(*ts):
    for t in ts:
        if t is not None and not t.is_cuda:
            raise ValueError("libsfl_sa kernels take device-resident tensors")


def as_u64(t: torch.Tensor) -> np.ndarray:
    """Host numpy uint64 view of a uint64-carrying int64 tensor."""
    return t.detach().cpu().numpy().view(np.uint64)


def xtype_of(dtype: torch.dtype) -> int:
    try:
        return _XTYPE[dtype]
    except KeyError:
        raise TypeError(f"unsupported element type {dtype}; use float32, float64 or int64") from None


def make_streams(entries: Sequence[tuple]) -> C.Array:
    """entries: (L.PCG64 gen, sign, peer) -> sa_mask_stream[]"""
    arr = (L.MaskStream * max(1, len(entries)))()
    for i, (g, sign, peer) in enumerate(entries):
        arr[i].gen = g
        arr[i].sign = int(sign)
        arr[i].peer = int(peer)
    return arr


def mask(x: torch.Tensor | None, out: torch.Tensor, streams: Sequence[tuple], *,
         weight: float = 1.0, weight_vec: torch.Tensor | None = None, compute_dtype=None,
         fxp_bits: int = 18, x_dtype=None, sum_accum: torch.Tensor | None = None,
         digest: torch.Tensor | None = None, flags: torch.Tensor | None = None) -> torch.Tensor:
    """One client's masked vector: out = trunc(x*w*2^fxp) +/- masks (mod 2^64).
    ``x=None`` continues from ``out`` (multi-pass).  See sa_mask in include/sfl_sa.h."""
    _require_gpu(x, out, weight_vec, sum_accum, digest, flags)
    n = out.numel()
    if x is not None and x.numel() != n:
        raise ValueError("x and out sizes differ")
    xt = xtype_of(x.dtype if x is not None else (x_dtype or torch.float32))
    ct = xtype_of(compute_dtype) if compute_dtype is not None else xt
    sarr = make_streams(streams)
    L.check(L.lib().sa_mask(_ptr(x), xt, ct, n, float(weight), _ptr(weight_vec), int(fxp_bits),
                            sarr, len(streams), _ptr(out), _ptr(sum_accum), _ptr(digest),
                            _ptr(flags), C.c_void_p(_stream(out))), "sa_mask")
    return out


def fused_clients(xs: Sequence[torch.Tensor], weights: Sequence[float], pair_gens: Sequence,
                  pair_signs: Sequence[int], cross: Sequence[tuple], n_cross: int,
                  sum_out: torch.Tensor, *, fxp_bits: int = 18, accumulate: bool = False,
                  digests: torch.Tensor | None = None, flags: torch.Tensor | None = None,
                  masked_outs: Sequence[torch.Tensor | None] | None = None) -> torch.Tensor:
    """C co-located clients in one launch: quantize, pairwise masks, masked sum.
    See sa_fused_clients in include/sfl_sa.h."""
    _require_gpu(sum_out, digests, flags, *xs)
    nc = len(xs)
    n = sum_out.numel()
    clients = (L.LocalClient * nc)()
    for c, x in enumerate(xs):
        if x.numel() != n or x.dtype != xs[0].dtype:
            raise ValueError("fused clients need equal-size vectors of one dtype")
        clients[c].x = x.data_ptr()
        clients[c].weight = float(weights[c])
        mo = masked_outs[c] if masked_outs else None
        clients[c].masked_out = mo.data_ptr() if mo is not None else None
    npair = nc * (nc - 1) // 2
    pg = (L.PCG64 * max(1, npair))(*pair_gens)
    ps = (C.c_int8 * max(1, npair))(*[int(s) for s in pair_signs])
    carr = make_streams(cross)
    rc = L.lib().sa_fused_clients(clients, nc, xtype_of(xs[0].dtype), n, int(fxp_bits), pg, ps,
                                  carr, int(n_cross), _ptr(sum_out), int(bool(accumulate)),
                                  _ptr(digests), _ptr(flags), C.c_void_p(_stream(sum_out)))
    if rc == L.SA_ERR_UNSUPPORTED:
        if (nc > 8 and n_cross == 0 and digests is None and not (masked_outs and any(m is not None for m in masked_outs))
                and xs[0].dtype == torch.float32):
            # more co-located clients than one launch holds, only the sum wanted:
            # the pair-shared schedule (every pair stream still expanded once)
            return fused_many(xs, weights, pair_gens, pair_signs, sum_out, fxp_bits=fxp_bits,
                              accumulate=accumulate, flags=flags)
        # other shapes without a fused instantiation (e.g. 32 clients, 4 per
        # GPU, with cross streams; or per-client digests / wire images): every
        # client masks with its own streams (both ends of each internal pair)
        # and accumulates into the sum -- same result, no pair sharing
        return _fused_fallback(xs, weights, pair_gens, pair_signs, cross, n_cross, sum_out, fxp_bits,
                               accumulate, digests, flags, masked_outs)
    L.check(rc, "sa_fused_clients")
    return sum_out


def many_schedule(nc: int) -> tuple[list[list[int]], list[tuple[list[int], list[int]]]]:
    """The pair-shared schedule of ``nc`` co-located clients (more than one
    launch holds): clients in quads of 4 (the last may be short), quads in
    groups of two.  Returns (groups, bipartite blocks): one sa_fused_clients
    launch per group (its clients' quantized values and every pair inside the
    group) and one sa_fused_bipartite launch per pair of quads in different
    groups (their cross pairs) -- every pair of clients exactly once."""
    quads = [list(range(q, min(nc, q + 4))) for q in range(0, nc, 4)]
    groups = [quads[g] + (quads[g + 1] if g + 1 < len(quads) else []) for g in range(0, len(quads), 2)]
    blocks = [(quads[a], quads[b]) for a in range(len(quads)) for b in range(a + 1, len(quads)) if a // 2 != b // 2]
    return groups, blocks


_PAD_STREAM = (0, 1)  # (state, inc) of a padding slot's pairs: drawn, and cancelled in the sum


def fused_many(xs: Sequence[torch.Tensor], weights: Sequence[float], pair_gens: Sequence, pair_signs: Sequence[int],
               sum_out: torch.Tensor, *, fxp_bits: int = 18, accumulate: bool = False,
               flags: torch.Tensor | None = None) -> torch.Tensor:
    """Masked sum of ``len(xs)`` co-located float32 clients (any number) with
    every pair stream expanded ONCE and applied to both of its clients
    (``many_schedule``; ``pair_gens`` / ``pair_signs`` in sa_fused_clients'
    u-major order).  All launches add into ``sum_out``; the sum equals the
    per-client path's bit for bit.  A short last quad is padded with slots
    that have no input and dummy pair streams, whose masks cancel in the sum."""
    _require_gpu(sum_out, flags, *xs)
    nc, n = len(xs), sum_out.numel()
    pidx, p = {}, 0
    for u in range(nc):
        for v in range(u + 1, nc):
            pidx[(u, v)] = p
            p += 1
    groups, blocks = many_schedule(nc)
    first = not accumulate
    for grp in groups:
        gp = [(u, v) for i, u in enumerate(grp) for v in grp[i + 1:]]
        fused_clients([xs[c] for c in grp], [weights[c] for c in grp], [pair_gens[pidx[q]] for q in gp],
                      [pair_signs[pidx[q]] for q in gp], [], 0, sum_out, fxp_bits=fxp_bits, accumulate=not first,
                      flags=flags)
        first = False
    pad = L.PCG64.of(*_PAD_STREAM)
    clients = (L.LocalClient * 8)()
    for c in range(8):
        clients[c].x, clients[c].weight, clients[c].masked_out = None, 1.0, None
    for qa, qb in blocks:
        gens, signs = [], []
        for i in range(4):
            for j in range(4):
                if i < len(qa) and j < len(qb):
                    q = pidx[(qa[i], qb[j])]
                    gens.append(pair_gens[q])
                    signs.append(int(pair_signs[q]))
                else:
                    gens.append(pad)
                    signs.append(1)
        L.check(L.lib().sa_fused_bipartite(clients, L.SA_F32, n, int(fxp_bits), (L.PCG64 * 16)(*gens),
                                           (C.c_int8 * 16)(*signs), _ptr(sum_out), 1, _ptr(flags),
                                           C.c_void_p(_stream(sum_out))), "sa_fused_bipartite")
    return sum_out


def _fused_fallback(xs, weights, pair_gens, pair_signs, cross, n_cross, sum_out, fxp_bits, accumulate,
                    digests, flags, masked_outs):
    nc = len(xs)
    per = [[] for _ in range(nc)]
    p = 0
    for u in range(nc):
        for v in range(u + 1, nc):
            per[u].append((pair_gens[p], int(pair_signs[p]), v))
            per[v].append((pair_gens[p], -int(pair_signs[p]), u))
            p += 1
    for c in range(nc):
        per[c].extend(cross[c * n_cross:(c + 1) * n_cross])
    if not accumulate:
        sum_out.zero_()
    scratch = None
    for c in range(nc):
        out = masked_outs[c] if masked_outs and masked_outs[c] is not None else None
        if out is None:
            scratch = scratch if scratch is not None else torch.empty_like(sum_out)
            out = scratch
        mask(xs[c], out, per[c], weight=weights[c], fxp_bits=fxp_bits, sum_accum=sum_out,
             digest=None if digests is None else digests[c:c + 1], flags=flags)
    return sum_out


def sum_u64(ins: Sequence[torch.Tensor], out: torch.Tensor) -> torch.Tensor:
    """Server sum mod 2^64 of masked vectors."""
    _require_gpu(out, *ins)
    n = out.numel()
    for t in ins:
        if t.numel() != n or t.device != out.device:
            raise ValueError("sum_u64 inputs must match out in size and device")
    ptrs = (C.c_void_p * len(ins))(*[t.data_ptr() for t in ins])
    L.check(L.lib().sa_sum_u64(ptrs, len(ins), n, _ptr(out), C.c_void_p(_stream(out))), "sa_sum_u64")
    return out


def decode(s: torch.Tensor, out: torch.Tensor, *, fxp_bits: int = 18, divisor: float = 1.0,
           divisor_vec: torch.Tensor | None = None) -> torch.Tensor:
    """float64 out = (int64)s / 2^fxp / divisor (or / divisor_vec[i])."""
    _require_gpu(s, out, divisor_vec)
    L.check(L.lib().sa_decode(_ptr(s), s.numel(), int(fxp_bits), float(divisor), _ptr(divisor_vec),
                              _ptr(out), C.c_void_p(_stream(out))), "sa_decode")
    return out


def host_fused_scratch(n_clients: int, n: int) -> tuple[int, int]:
    """(pinned bytes, device bytes) sa_fused_clients_host_f32 needs."""
    n_pad, meta = -(-n // 4) * 4, (n_clients + 2) // 2 * 2  # flag + digests, an even word count
    pin = n_clients * n_pad * 4 + (meta + n_pad) * 8
    return pin, pin + n_pad * 8


def fused_clients_host_f32(xs: Sequence[np.ndarray], weights: Sequence[float], pair_gens: Sequence,
                           pair_signs: Sequence[int], pinned: torch.Tensor, dev: torch.Tensor, *,
                           fxp_bits: int = 18, divisor: float = 1.0):
    """Host float32 vectors of 2..8 co-located clients -> (decoded float64
    host array, uint64 digests, flag word) in ONE blocking call (see
    sa_fused_clients_host_f32 in include/sfl_sa.h).  ``pinned`` / ``dev``:
    byte tensors of host_fused_scratch's sizes (page-locked / on the GPU).
    None when the library has no fused kernel for this client count."""
    _require_gpu(dev)
    nc, n = len(xs), int(xs[0].size)
    need_pin, need_dev = host_fused_scratch(nc, n)
    if not pinned.is_pinned() or pinned.numel() < need_pin or dev.numel() < need_dev:
        raise ValueError("scratch buffers too small or not page-locked")
    arrs = [np.ascontiguousarray(x, dtype=np.float32).reshape(-1) for x in xs]
    if any(a.size != n for a in arrs):
        raise ValueError("fused clients need equal-size vectors")
    ptrs = (C.c_void_p * nc)(*[a.ctypes.data for a in arrs])
    ws = (C.c_double * nc)(*[float(w) for w in weights])
    npair = nc * (nc - 1) // 2
    pg = (L.PCG64 * max(1, npair))(*pair_gens)
    ps = (C.c_int8 * max(1, npair))(*[int(s) for s in pair_signs])
    out = np.empty(n, dtype=np.float64)
    digests = np.empty(nc, dtype=np.uint64)
    flags = C.c_uint32(0)
    rc = L.lib().sa_fused_clients_host_f32(ptrs, ws, nc, n, int(fxp_bits), pg, ps, float(divisor),
                                           _ptr(pinned), _ptr(dev), C.c_void_p(out.ctypes.data),
                                           C.c_void_p(digests.ctypes.data), C.byref(flags),
                                           C.c_void_p(_stream(dev)))
    if rc == L.SA_ERR_UNSUPPORTED:
        return None
    L.check(rc, "sa_fused_clients_host_f32")
    return out, digests, int(flags.value)


_NP_XTYPE = {np.dtype(np.float32): L.SA_F32, np.dtype(np.float64): L.SA_F64, np.dtype(np.int64): L.SA_I64}


def host_clients_scratch(n_clients: int, n: int, itemsize: int) -> tuple[int, int]:
    """(pinned bytes, device bytes) sa_clients_host needs."""
    n_pad, meta = -(-n // 4) * 4, (n_clients + 2) // 2 * 2
    pin = n_clients * n_pad * itemsize + (2 * n_pad + meta) * 8
    return pin, pin + n_clients * n_pad * 8


def clients_host(xs: Sequence[np.ndarray], compute_dtype, weights: Sequence[float], streams: Sequence[Sequence],
                 pinned: torch.Tensor, dev: torch.Tensor, *, fxp_bits: int = 18, divisor: float = 1.0):
    """Host vectors of one element type (float32 / float64 / int64) of 2..9
    co-located clients, each masked with its own streams (``streams[c]``:
    (gen, sign, peer) triples) -> (decoded float64 host array, uint64
    digests, flag word) in ONE blocking call (sa_clients_host in
    include/sfl_sa.h)."""
    _require_gpu(dev)
    nc, n = len(xs), int(np.asarray(xs[0]).size)
    dt = np.asarray(xs[0]).dtype
    arrs = [np.ascontiguousarray(x, dtype=dt).reshape(-1) for x in xs]
    if dt not in _NP_XTYPE or any(a.size != n for a in arrs):
        raise ValueError("host clients need equal-size float32 / float64 / int64 vectors of one type")
    need_pin, need_dev = host_clients_scratch(nc, n, dt.itemsize)
    if not pinned.is_pinned() or pinned.numel() < need_pin or dev.numel() < need_dev:
        raise ValueError("scratch buffers too small or not page-locked")
    if any(len(st) != nc - 1 for st in streams):
        raise ValueError("every client needs n_clients - 1 streams")
    ptrs = (C.c_void_p * nc)(*[a.ctypes.data for a in arrs])
    ws = (C.c_double * nc)(*[float(w) for w in weights])
    sarr = make_streams([e for st in streams for e in st])
    out = np.empty(n, dtype=np.float64)
    digests = np.empty(nc, dtype=np.uint64)
    flags = C.c_uint32(0)
    ct = _NP_XTYPE[np.dtype(compute_dtype)]
    L.check(L.lib().sa_clients_host(ptrs, _NP_XTYPE[dt], ct, ws, nc, n, int(fxp_bits), sarr, float(divisor),
                                    _ptr(pinned), _ptr(dev), C.c_void_p(out.ctypes.data),
                                    C.c_void_p(digests.ctypes.data), C.byref(flags), C.c_void_p(_stream(dev))),
            "sa_clients_host")
    return out, digests, int(flags.value)


def _scratch(pinned: torch.Tensor, dev: torch.Tensor, need_pin: int, need_dev: int) -> None:
    _require_gpu(dev)
    if not pinned.is_pinned() or pinned.numel() < need_pin or dev.numel() < need_dev:
        raise ValueError("scratch buffers too small or not page-locked")


def mask_host_scratch(n: int, itemsize: int) -> tuple[int, int]:
    """(pinned bytes, device bytes) sa_mask_host needs."""
    n_pad = -(-n // 4) * 4
    return n_pad * itemsize + (2 + n_pad) * 8, n_pad * itemsize + (2 + n_pad) * 8


def mask_host(x: np.ndarray, compute_dtype, streams: Sequence[tuple], pinned: torch.Tensor, dev: torch.Tensor, *,
              weight: float = 1.0, fxp_bits: int = 18):
    """One party's masked vector from a host array in ONE blocking call
    (sa_mask_host in include/sfl_sa.h) -> (uint64 host array, flag word)."""
    a = np.ascontiguousarray(x).reshape(-1)
    if a.dtype not in _NP_XTYPE:
        raise ValueError("mask_host takes float32 / float64 / int64 host arrays")
    n = int(a.size)
    _scratch(pinned, dev, *mask_host_scratch(n, a.dtype.itemsize))
    sarr = make_streams(streams)
    out = np.empty(n, dtype=np.uint64)
    flags = C.c_uint32(0)
    L.check(L.lib().sa_mask_host(C.c_void_p(a.ctypes.data), _NP_XTYPE[a.dtype], _NP_XTYPE[np.dtype(compute_dtype)],
                                 n, float(weight), int(fxp_bits), sarr, len(streams), _ptr(pinned), _ptr(dev),
                                 C.c_void_p(out.ctypes.data), C.byref(flags), C.c_void_p(_stream(dev))),
            "sa_mask_host")
    return out, int(flags.value)


def sum_decode_host_scratch(n_clients: int, n: int) -> tuple[int, int]:
    """(pinned bytes, device bytes) sa_sum_decode_host needs."""
    n_pad, meta = -(-n // 4) * 4, (n_clients + 1) // 2 * 2
    pin = (n_clients * n_pad + meta + n_pad) * 8
    return pin, pin + n_pad * 8


def sum_decode_host(masked: Sequence[np.ndarray], pinned: torch.Tensor, dev: torch.Tensor, *, fxp_bits: int = 18,
                    divisor: float = 1.0):
    """The server's step on host masked vectors in ONE blocking call
    (sa_sum_decode_host in include/sfl_sa.h) -> (decoded float64 host array,
    uint64 digests as received)."""
    arrs = [np.ascontiguousarray(m).view(np.uint64).reshape(-1) for m in masked]
    nc, n = len(arrs), int(arrs[0].size)
    if any(a.size != n for a in arrs):
        raise ValueError("masked vectors of different sizes")
    _scratch(pinned, dev, *sum_decode_host_scratch(nc, n))
    ptrs = (C.c_void_p * nc)(*[a.ctypes.data for a in arrs])
    out = np.empty(n, dtype=np.float64)
    digests = np.empty(nc, dtype=np.uint64)
    L.check(L.lib().sa_sum_decode_host(ptrs, nc, n, int(fxp_bits), float(divisor), _ptr(pinned), _ptr(dev),
                                       C.c_void_p(out.ctypes.data), C.c_void_p(digests.ctypes.data),
                                       C.c_void_p(_stream(dev))), "sa_sum_decode_host")
    return out, digests


def sum_f64(ins: Sequence[torch.Tensor], out: torch.Tensor) -> torch.Tensor:
    _require_gpu(out, *ins)
    ptrs = (C.c_void_p * len(ins))(*[t.data_ptr() for t in ins])
    L.check(L.lib().sa_sum_f64(ptrs, len(ins), out.numel(), _ptr(out), C.c_void_p(_stream(out))),
            "sa_sum_f64")
    return out


# ---------------------------------------------------------------------------
# GaussianModelDP pre-step (sa_sumsq_f32 / sa_dp_perturb_f32 / sa_mask_dp)
# ---------------------------------------------------------------------------
def make_dp(sumsq: torch.Tensor, *, l2_norm_clip: float, noise_std: float, num_updates: float, key: int,
            counter0: int = 0, sumsq_layer: torch.Tensor | None = None) -> L.DP:
    if counter0 % 4:
        raise ValueError("counter0 must be a multiple of 4")
    d = L.DP()
    d.sumsq = sumsq.data_ptr()
    d.sumsq_layer = sumsq_layer.data_ptr() if sumsq_layer is not None else None
    d.l2_norm_clip = float(l2_norm_clip)
    d.noise_std = float(noise_std)
    d.num_updates = float(num_updates)
    d.key = int(key) & ((1 << 64) - 1)
    d.counter0 = int(counter0)
    return d


def sumsq_f32(x: torch.Tensor, out: torch.Tensor, partials: torch.Tensor, *, accumulate: bool = False) -> torch.Tensor:
    """out[0] (+)= the layer's squared norm as the reference forms it (the
    float32 np.linalg.norm, squared in float64; sa_sumsq_f32)."""
    _require_gpu(x, out, partials)
    if x.dtype != torch.float32 or out.dtype != torch.float64 or partials.numel() < L.SA_DP_PARTIALS:
        raise ValueError("sumsq_f32: float32 x, float64 out, SA_DP_PARTIALS float64 partials")
    L.check(L.lib().sa_sumsq_f32(_ptr(x), x.numel(), _ptr(partials), _ptr(out), int(bool(accumulate)),
                                 C.c_void_p(_stream(out))), "sa_sumsq_f32")
    return out


def dp_perturb(x: torch.Tensor, out: torch.Tensor, dp: L.DP) -> torch.Tensor:
    _require_gpu(x, out)
    if x.dtype != torch.float32 or out.dtype != torch.float32 or out.numel() != x.numel():
        raise ValueError("dp_perturb: float32 x and out of equal size")
    L.check(L.lib().sa_dp_perturb_f32(_ptr(x), x.numel(), C.byref(dp), _ptr(out), C.c_void_p(_stream(out))),
            "sa_dp_perturb_f32")
    return out


def mask_dp(x: torch.Tensor, out: torch.Tensor, streams: Sequence[tuple], dp: L.DP, *, weight: float = 1.0,
            fxp_bits: int = 18, sum_accum: torch.Tensor | None = None, digest: torch.Tensor | None = None,
            flags: torch.Tensor | None = None) -> torch.Tensor:
    """sa_mask of the DP-perturbed float32 x, perturbation fused into the kernel."""
    _require_gpu(x, out, sum_accum, digest, flags)
    if x.dtype != torch.float32 or x.numel() != out.numel():
        raise ValueError("mask_dp: float32 x with out of equal size")
    sarr = make_streams(streams)
    L.check(L.lib().sa_mask_dp(_ptr(x), x.numel(), float(weight), int(fxp_bits), sarr, len(streams), C.byref(dp),
                               _ptr(out), _ptr(sum_accum), _ptr(digest), _ptr(flags), C.c_void_p(_stream(out))),
            "sa_mask_dp")
    return out


# ---------------------------------------------------------------------------
# numpy's rejection re-draw (after SA_FLAG_PRG_REJECT; never on the hot path)
# ---------------------------------------------------------------------------
U64_MAX = (1 << 64) - 1


def find_zero_draws(gens: Sequence, n: int, device) -> list:
    """For each generator, the first raw draw index in [0, n) whose PCG64
    output is 0 (numpy's Generator.integers rejects it), or None."""
    if not gens:
        return []
    first = torch.full((len(gens),), -1, dtype=torch.int64, device=device)  # all ones = UINT64_MAX
    arr = (L.PCG64 * len(gens))(*gens)
    L.check(L.lib().sa_pcg64_find_zero(arr, len(gens), int(n), _ptr(first), C.c_void_p(_stream(first))),
            "sa_pcg64_find_zero")
    return [None if v == U64_MAX else int(v) for v in as_u64(first).tolist()]


def stream_shift(out: torch.Tensor, gen, sign: int, k: int, shift: int) -> torch.Tensor:
    """out[e] += sign * (raw[e+shift] - raw[e+shift-1]) for e >= k (in place)."""
    _require_gpu(out)
    g = L.PCG64(gen.state, gen.inc)
    L.check(L.lib().sa_stream_shift(_ptr(out), out.numel(), C.byref(g), int(sign), int(k), int(shift),
                                    C.c_void_p(_stream(out))), "sa_stream_shift")
    return out


def xor_digest(v: torch.Tensor, digest: torch.Tensor) -> torch.Tensor:
    """digest[0] ^= XOR of every uint64 element of v."""
    _require_gpu(v, digest)
    L.check(L.lib().sa_xor_u64(_ptr(v), v.numel(), _ptr(digest), C.c_void_p(_stream(v))), "sa_xor_u64")
    return digest


def rejected_draws(gen, n: int, device, first: int | None = -1) -> tuple[list, int]:
    """numpy's Generator.integers over n elements from ``gen``: the
    (element, shift) points where a rejected raw 0 moves the stream one raw
    draw further (element e >= k uses raw[e + shift]), and the total number
    of raw draws consumed (n + rejections).  ``first``: the stream's first
    zero in [0, n) when already searched (None: there is none)."""
    if first is None:
        return [], n
    pts, e0, s = [], 0, 0
    if first != -1:
        e0, s = first, 1
        pts.append((e0, s))
    while e0 < n:
        # elements >= e0 use raw[e + s]: search raw[e0 + s, n + s)
        z = find_zero_draws([L.pcg64_advance(gen, e0 + s)], n - e0, device)[0]
        if z is None:
            break
        e0, s = e0 + z, s + 1
        pts.append((e0, s))
    return pts, n + s


def rejected_draws_many(gens: Sequence, n: int, device) -> list:
    """``rejected_draws`` for many streams: the first zero of every stream is
    searched by ONE sa_pcg64_find_zero call (up to 64 generators per launch
    inside it) and one host sync; only the streams with a hit are followed
    further."""
    first = find_zero_draws(list(gens), n, device)
    return [rejected_draws(g, n, device, first=f) for g, f in zip(gens, first)]
