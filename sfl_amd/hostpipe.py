"""Host-array <-> GPU pipelining for the drop-in's large payloads.

A party's ``mask_payload`` and the server's ``sum_decode`` start and end in
host memory (numpy arrays a secretflow PYU hands over and ships on).  For a
large payload the time is the PCIe copies (``tools/pcie_paths.py`` on
MI355X: ~57 GB/s each way, ~79 GB/s both ways at once), not the kernels (a
100M-element party mask is ~0.5 ms of device time).  So:

* the element range is cut into chunks; chunk j's H2D, its kernels and its
  D2H run on three streams ordered by events, overlapping chunk j+1's;
* every DMA touches page-locked memory only: the caller's arrays are
  registered for the call (``Pinned``; chunk by chunk as their copies are
  issued, ``Issued``), or, where the driver refuses that, staged through
  pinned slots (torch's caching host allocator) by a feeder thread whose
  memcpy runs on a thread pool (75-97 GB/s on 8-16 threads, above the PCIe
  rate, tools/pcie_paths.py); no copy is pageable (pageable D2H copies into
  fresh arrays beside registered memory failed now and then with
  hipErrorInvalidValue, once aborting in the next synchronise, and once
  with an illegal address: ``d2h`` / ``h2d`` serve the one-shot paths);
* the result goes into a recycled registered buffer (``ResultPool``: free
  once the caller dropped every array viewing it), so its D2H is async DMA
  into pages that are in; on a miss, chunk j lands in a pinned slot and a
  drain thread copies it into a fresh ``np.empty`` (faulting its pages on
  the pool's threads) while chunk j+1 is in flight.

Nothing here computes: the kernels are the library's (``sa_mask``,
``sa_xor_u64``, ``sa_sum_u64``, ``sa_decode``, ``sa_fused_clients``).  Used
by ``security/aggregation/party.py`` and ``secure_aggregator.py``.
"""

from __future__ import annotations

import bisect
import ctypes
import os
import queue
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

_POOL = None
# SFL_HOSTPIPE_TRACE=1: every pipelined call prints its phase times to stderr
TRACE = os.environ.get("SFL_HOSTPIPE_TRACE") == "1"
_POOL_LOCK = threading.Lock()
COPY_THREADS = 12  # of the box's 16-CPU share: the feeder, the drain and the caller keep the rest
PAGE = 4096
SLOTS = 3  # pinned staging slots per direction and call


def _pool() -> ThreadPoolExecutor:
    """Leaf tasks only (memcpy pieces, page touches): nothing submitted
    here waits on another task of this pool."""
    global _POOL
    with _POOL_LOCK:
        if _POOL is None:
            _POOL = ThreadPoolExecutor(COPY_THREADS, thread_name_prefix="sfl_sa_copy")
    return _POOL


def pcopy(dst: np.ndarray, src: np.ndarray) -> None:
    """dst[:] = src (same shape, contiguous), in pieces of >= 1 MiB on the
    pool's threads (numpy's copy releases the GIL)."""
    nb = dst.nbytes
    k = min(COPY_THREADS, max(1, nb >> 20))
    if k == 1:
        np.copyto(dst, src)
        return
    step = -(-dst.size // k)
    list(_pool().map(lambda a: np.copyto(dst[a:a + step], src[a:a + step]), range(0, dst.size, step)))


# chunks per pipelined call (SFL_HOSTPIPE_CHUNKS; a party's mask_payload asks for 16 itself)
CHUNKS = int(os.environ.get("SFL_HOSTPIPE_CHUNKS", "8"))


def chunk_bounds(n: int, target: int | None = None, lo_elems: int = 1 << 20, hi_elems: int = 1 << 24,
                 align: int = 1024) -> list[tuple[int, int]]:
    """[0, n) in about ``target`` (default ``CHUNKS``) chunks of
    lo_elems..hi_elems elements, each start a multiple of ``align`` (16-byte
    aligned device slices)."""
    if n <= 0:
        return []
    target = CHUNKS if target is None else target
    step = min(max(-(-n // target), lo_elems), hi_elems)
    step = -(-step // align) * align
    return [(lo, min(n, lo + step)) for lo in range(0, n, step)]


_NP_OF = {"torch.float32": np.float32, "torch.float64": np.float64, "torch.float16": np.float16,
          "torch.int64": np.int64, "torch.int32": np.int32, "torch.uint8": np.uint8, "torch.bool": np.bool_}


def host_dtype(t):
    """The numpy dtype ``d2h`` gives tensor ``t``'s elements (None: numpy has none, e.g. bfloat16)."""
    dt = _NP_OF.get(str(t.dtype))
    return None if dt is None else np.dtype(dt)


def d2h(t, pooled: bool = True) -> np.ndarray:
    """A device tensor's elements in a new host array without a pageable
    DMA (a large pageable copy beside registered memory -- ``RESULTS``,
    ``Pinned`` -- failed now and then with hipErrorInvalidValue or an
    illegal address; every host copy of the one-shot paths goes through
    here): straight into a recycled registered buffer when ``pooled`` and
    one is free, else into a pinned buffer and out of it on the pool's
    threads.  Blocking."""
    import torch

    t = t.detach().contiguous()
    dt = host_dtype(t)
    if dt is None:
        raise TypeError(f"no host array type for {t.dtype}")
    nb = t.numel() * t.element_size()
    owner = RESULTS.take(nb) if pooled else None
    if owner is not None:
        out = owner[:nb].view(dt)
        torch.from_numpy(out).copy_(t.reshape(-1))
        return out.reshape(tuple(t.shape))
    h = torch.empty(t.numel(), dtype=t.dtype, pin_memory=True)
    h.copy_(t.reshape(-1))
    out = np.empty(t.numel(), dt)
    pcopy(out, h.numpy())
    return out.reshape(tuple(t.shape))


def h2d(a, dev):
    """A host array (numpy or a CPU tensor) as a new tensor on ``dev``,
    without a pageable DMA (``d2h``): an array inside a pooled result is
    copied as it is (registered), anything else through a pinned buffer
    filled on the pool's threads.  Ordered on ``dev``'s current stream."""
    import torch

    if isinstance(a, torch.Tensor):
        if a.device.type != "cpu":
            return a.detach().to(dev)
        a = a.detach().numpy()
    a = np.ascontiguousarray(a).reshape(np.shape(a))  # (ascontiguousarray makes a 0-d array 1-d)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    if a.size == 0:
        return torch.from_numpy(a).to(dev)
    if RESULTS.contains(a):
        return _tensor(a).to(dev)
    h = torch.empty(a.shape, dtype=_tensor(a.reshape(-1)[:0]).dtype, pin_memory=True)
    pcopy(h.numpy().reshape(-1), a.reshape(-1))
    return h.to(dev, non_blocking=True)


def page_bounds(bounds: list[tuple[int, int]], layer_lists) -> list[tuple[int, int]]:
    """``bounds`` with each chunk join moved up by less than a page of
    elements onto a page boundary of every party's layer holding it, where
    one such move exists (the parties' arrays share their offset within a
    page, as numpy's large allocations do), the join stays at a 16-byte
    multiple (aligned device slices: the kernels' requirement) and inside
    its layer.  Lazily registered inputs (``Pinned``) then register exactly
    chunk by chunk and no copy is cut.  ``layer_lists``: per party, its flat
    layers (same sizes and element type for every party)."""
    if len(bounds) < 2 or not layer_lists:
        return bounds
    sizes = [a.size for a in layer_lists[0]]
    if any([a.size for a in ll] != sizes for ll in layer_lists[1:]):
        return bounds
    isz = layer_lists[0][0].itemsize
    starts = np.cumsum([0] + sizes).tolist()
    out = [list(b) for b in bounds]
    for k in range(1, len(bounds)):
        lo = bounds[k][0]
        li = bisect.bisect_right(starts, lo) - 1
        need = {-(ll[li].ctypes.data + (lo - starts[li]) * isz) % PAGE for ll in layer_lists}
        if len(need) != 1:
            continue
        nb = need.pop()
        new = lo + nb // isz
        if nb % isz or new * isz % 16 or new >= starts[li + 1] or new >= bounds[k][1]:
            continue
        out[k - 1][1] = out[k][0] = new
    return [tuple(b) for b in out]


class Slots:
    """``SLOTS`` page-locked staging buffers of ``nbytes`` each, used round
    robin; ``take(k)`` waits until slot k's previous use is over (a device
    event: its DMA; or a threading.Event: the host copy out of it)."""

    def __init__(self, nbytes: int, n: int = SLOTS):
        import torch

        self.bufs = [torch.empty(max(nbytes, 16), dtype=torch.uint8, pin_memory=True) for _ in range(n)]
        self.busy = [None] * n

    def take(self, k: int):
        k %= len(self.bufs)
        b = self.busy[k]
        if isinstance(b, threading.Event):
            b.wait()
        elif b is not None:
            b.synchronize()
        return k, self.bufs[k]

    def release(self, k: int, until) -> None:
        self.busy[k] = until

    def drain(self) -> None:
        for k in range(len(self.bufs)):
            self.take(k)
            self.busy[k] = None


def _np(t, dtype) -> np.ndarray:
    return t.numpy().view(np.dtype(dtype))


class FreshOutput:
    """A host result of ``n`` elements that the device fills chunk by chunk.
    A recycled registered buffer from ``RESULTS`` when one is free: chunk
    j's D2H is async DMA straight into it.  Otherwise a fresh ``np.empty``
    (numpy advises huge pages for large allocations: first touch ~27 GB/s a
    thread against ~8 GB/s for a plain anonymous mmap, tools/touch_probe.py)
    that chunk j reaches through a pinned slot: DMA into the slot, then the
    drain thread copies the slot out on the pool's threads while later
    chunks are in flight.  ``array`` is the caller's result; ``close()``
    waits for the drain."""

    def __init__(self, n: int, dtype, bounds):
        dtype = np.dtype(dtype)
        self.dtype, self.bounds = dtype, bounds
        self.stats = {"pooled": False, "drain_ms": 0.0}
        self._q = self._thread = self._error = None
        owner = RESULTS.take(n * dtype.itemsize)
        if owner is not None:  # a recycled, registered buffer: no faults, async DMA
            self.array = owner[:n * dtype.itemsize].view(dtype)
            self.stats["pooled"] = True
            return
        self.array = np.empty(n, dtype=dtype)
        chunk = max((hi - lo for lo, hi in bounds), default=0)
        self._slots = Slots(chunk * dtype.itemsize)
        self._q = queue.Queue()
        self._thread = threading.Thread(target=self._drain, name="sfl_sa_d2h", daemon=True)
        self._thread.start()

    def _drain(self) -> None:
        while True:
            item = self._q.get()
            if item is None:
                return
            j, k, ev, done = item
            try:
                if self._error is None:
                    t0 = time.perf_counter()
                    ev.synchronize()
                    lo, hi = self.bounds[j]
                    pcopy(self.array[lo:hi], _np(self._slots.bufs[k], self.dtype)[:hi - lo])
                    self.stats["drain_ms"] += 1e3 * (time.perf_counter() - t0)
            except BaseException as ex:  # noqa: BLE001 - re-raised by close()
                self._error = ex
            finally:
                done.set()

    def copy_in(self, j: int, src, stream, after) -> None:
        """D2H of chunk j: ``src`` (a device tensor of chunk j's elements)
        into this result on ``stream`` once event ``after`` has passed."""
        import torch

        lo, hi = self.bounds[j]
        with torch.cuda.stream(stream):
            stream.wait_event(after)
            if self.stats["pooled"]:
                dst = self.array[lo:hi]
                torch.from_numpy(dst.view(np.int64) if dst.dtype == np.uint64 else dst).copy_(src, non_blocking=True)
                return
            k, slot = self._slots.take(j)
            nb = (hi - lo) * self.dtype.itemsize
            slot[:nb].view(src.dtype).copy_(src, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
        done = threading.Event()  # set by the drain once the slot is copied out
        self._slots.release(k, done)
        self._q.put((j, k, ev, done))

    def close(self) -> None:
        if self._thread is not None:
            self._q.put(None)
            self._thread.join()
            self._thread = None
            if self._error is not None:
                raise self._error


class ResultPool:
    """Registered host buffers for the pipelined results, recycled once the
    caller has dropped every array that views them: a per-party masked
    vector is shipped and dropped every round, so from the second round on
    its D2H lands in registered pages without a fault (the fresh-result path
    pays ~6 ms of page faults and a pageable copy per 800 MB).  A buffer is
    free when nothing but the pool references it (``sys.getrefcount``: every
    numpy view of it holds its owner).  New buffers are made on a miss while
    the pool holds less than ``cap`` bytes (SFL_HOSTPIPE_POOL_BYTES, default
    8 GiB; 0 disables), at the cost of one fresh result (parallel first
    touch, then one registration); beyond the cap, results are fresh arrays
    again."""

    def __init__(self, cap: int):
        self.cap = cap
        self.bufs: list = []
        self.lock = threading.Lock()

    def take(self, nbytes: int):
        if nbytes < (8 << 20) or self.cap <= 0:
            return None
        with self.lock:
            best = None
            for i in range(len(self.bufs)):
                if self.bufs[i].nbytes >= nbytes and sys.getrefcount(self.bufs[i]) == 2:
                    if best is None or self.bufs[i].nbytes < self.bufs[best].nbytes:
                        best = i
            if best is not None:
                return self.bufs[best]
            if sum(b.nbytes for b in self.bufs) + nbytes > self.cap:
                return None
            owner = np.empty(nbytes, dtype=np.uint8)
            step = -(-nbytes // COPY_THREADS) // PAGE * PAGE + PAGE

            def touch(lo):
                owner[lo:lo + step:PAGE] = 0

            list(_pool().map(touch, range(0, nbytes, step)))
            hip = _hip()
            if hip.hipHostRegister(ctypes.c_void_p(owner.ctypes.data), ctypes.c_size_t(nbytes), ctypes.c_uint(0)):
                hip.hipGetLastError()
                return None
            self.bufs.append(owner)
            return owner

    def contains(self, a: np.ndarray) -> bool:
        """``a``'s memory lies inside one of the pool's (registered) buffers."""
        p0, p1 = a.ctypes.data, a.ctypes.data + a.nbytes
        with self.lock:
            return any(b.ctypes.data <= p0 and p1 <= b.ctypes.data + b.nbytes for b in self.bufs)

    def clear(self) -> None:
        """Unregister and drop every free buffer (tests, memory pressure)."""
        with self.lock:
            keep = []
            for i in range(len(self.bufs)):
                if sys.getrefcount(self.bufs[i]) == 2:
                    _hip().hipHostUnregister(ctypes.c_void_p(self.bufs[i].ctypes.data))
                else:
                    keep.append(self.bufs[i])
            self.bufs = keep


RESULTS = ResultPool(int(os.environ.get("SFL_HOSTPIPE_POOL_BYTES", str(8 << 30))))


class Feeder:
    """The H2D side of a pipelined call, on a helper thread.  ``chunks[j]``
    lists chunk j's copies as (device tensor slice, pieces): ``pieces`` are
    (host array, element offset in the slice) covering the slice.  Each
    copy is staged through a pinned slot (memcpy on the pool's threads, the
    DMA async on ``stream``); ``ready(j)`` returns the device event chunk j's
    copies complete at, once they are issued."""

    def __init__(self, stream, chunks):
        import torch

        self.stream, self.chunks = stream, chunks
        self.flags = [threading.Event() for _ in chunks]
        self.events = [None] * len(chunks)
        self.error = None
        nb = max((d.numel() * d.element_size() for ch in chunks for d, _ in ch), default=0)
        self.slots = Slots(nb)
        self._dt = {torch.float32: np.float32, torch.float64: np.float64, torch.int64: np.int64}
        self.thread = threading.Thread(target=self._run, name="sfl_sa_h2d", daemon=True)
        self.thread.start()

    def _run(self) -> None:
        import torch

        try:
            with torch.cuda.device(self.stream.device), torch.cuda.stream(self.stream):
                n = 0
                for j, chunk in enumerate(self.chunks):
                    for dst, pieces in chunk:
                        k, slot = self.slots.take(n)
                        n += 1
                        nb = dst.numel() * dst.element_size()
                        view = _np(slot, self._dt[dst.dtype])[:dst.numel()]
                        for a, off in pieces:
                            pcopy(view[off:off + a.size], a)
                        dst.copy_(slot[:nb].view(dst.dtype), non_blocking=True)
                        e = torch.cuda.Event()
                        e.record(self.stream)
                        self.slots.release(k, e)
                    e = torch.cuda.Event()
                    e.record(self.stream)
                    self.events[j] = e
                    self.flags[j].set()
        except BaseException as ex:  # noqa: BLE001 - re-raised in the caller's thread
            self.error = ex
            for f in self.flags:
                f.set()

    def ready(self, j: int):
        self.flags[j].wait()
        if self.error is not None:
            raise self.error
        return self.events[j]

    def join(self, check: bool = True) -> None:
        """Wait for the thread; with ``check``, re-raise its error here."""
        self.thread.join()
        if check and self.error is not None:
            raise self.error


class Issued:
    """``Feeder``'s interface for inputs that are registered for the call
    (``Pinned``): chunk j's copies, async DMA straight from the caller's
    pages, issued from the calling thread when ``ready(j)`` is first asked
    for, with chunk j+1's behind them.  Not all at once: a stream holds a
    bounded number of outstanding copies, and issuing config 5's 512 copies
    up front blocked the caller until most had finished, so no launch
    overlapped them.  With a lazily registering ``pin``, each piece is
    registered just before its copy is issued (``Pinned.split``), so the
    registration of chunk j+1 runs while chunk j's DMA is in flight."""

    LOOKAHEAD = int(os.environ.get("SFL_HOSTPIPE_LOOKAHEAD", "1"))  # chunks issued ahead of the one asked for

    def __init__(self, stream, chunks, pin=None):
        self.stream, self.chunks = stream, chunks
        self.pin = pin if pin is not None and pin.spans else None
        self.events = []

    def _issue(self, j: int) -> None:
        import torch

        with torch.cuda.stream(self.stream):
            for dst, pcs in self.chunks[j]:
                for a, off in pcs:
                    d = dst[off:off + a.size]
                    if self.pin is None:
                        d.copy_(_tensor(a), non_blocking=True)
                        continue
                    db, ab = d.view(torch.uint8), a.view(np.uint8)
                    for b0, b1, registered in self.pin.split(a):
                        if registered:
                            db[b0:b1].copy_(_tensor(ab[b0:b1]), non_blocking=True)
                        else:  # the driver refused this range: a pinned temporary (kept until its DMA is done)
                            tmp = torch.empty(b1 - b0, dtype=torch.uint8, pin_memory=True)
                            pcopy(tmp.numpy(), ab[b0:b1])
                            db[b0:b1].copy_(tmp, non_blocking=True)
            e = torch.cuda.Event()
            e.record(self.stream)
            self.events.append(e)

    def ready(self, j: int):
        while len(self.events) <= min(j + self.LOOKAHEAD, len(self.chunks) - 1):
            self._issue(len(self.events))
        return self.events[j]

    def join(self, check: bool = True) -> None:
        pass


def _tensor(a: np.ndarray):
    import warnings

    import torch

    with warnings.catch_warnings():  # a read-only caller array is only read here
        warnings.filterwarnings("ignore", message="The given NumPy array is not writable")
        return torch.from_numpy(a)


# SFL_HOSTPIPE_REGISTER=0: never register the caller's inputs (the feeder
# stages every one that is not a pooled result)
REGISTER = os.environ.get("SFL_HOSTPIPE_REGISTER", "1") != "0"
# SFL_HOSTPIPE_LAZY_REGISTER=0: register every large input whole on entry
# instead of piece by piece as its copies are issued
LAZY_REGISTER = os.environ.get("SFL_HOSTPIPE_LAZY_REGISTER", "1") != "0"
LAZY_MIN_BYTES = 64 << 20  # smaller arrays are registered whole on entry
# each lazy registration covers at least LAZY_GROWTH x what the array has
# registered so far (1: exactly what the copy at hand needs)
LAZY_GROWTH = int(os.environ.get("SFL_HOSTPIPE_LAZY_GROWTH", "2"))


class _Span:
    """A lazily registered array: its bytes [start, end), registered from
    ``base`` (its first page) up to ``reg_end``, the registrations' joins,
    and whether the driver refused a registration (the rest is staged)."""

    __slots__ = ("start", "end", "base", "reg_end", "cap", "joins", "refused")

    def __init__(self, p0: int, p1: int):
        self.start, self.end = p0, p1
        self.base = self.reg_end = p0 // PAGE * PAGE
        self.cap = -(-p1 // PAGE) * PAGE
        self.joins, self.refused = [], False


class Pinned:
    """hipHostRegister a party's input layers for a ``with`` block, so their
    H2D is async DMA issued from the calling thread (``Issued``) instead of
    staged by the feeder: the party's 400 MB in then overlaps its 800 MB out
    completely (16.3 against ~27 ms for 100M floats).  Only our own copies
    touch these pages while they are registered, and none of them is
    pageable.  Arrays inside a pooled result (``RESULTS``: e.g. the masked
    vectors the server receives from parties in the same process) are
    registered already and taken as they are; with ``register=False``
    nothing else is registered (``ok`` then says whether every array was
    pooled).  ``ok`` is False when the driver refuses an array registered
    on entry (already registered elsewhere, or sharing a page with
    registered memory): nothing stays registered and the caller stages
    through the feeder.  Unregistered on exit.

    Lazily (``LAZY_REGISTER``, arrays of ``LAZY_MIN_BYTES`` or more):
    nothing is registered on entry; ``split`` registers an array's pages as
    ``Issued`` reaches them, each time at least ``LAZY_GROWTH`` x what it
    holds already (chunk 0, then 1, then 2-3, 4-7, ...: few calls, ~0.1-0.2
    ms each whatever their size), so registering 32 GB of config-5 inputs
    (57 ms before the first copy) overlaps the copies of earlier chunks.  A
    copy never spans two registrations: ``split`` cuts it at their joins.
    A registration the driver refuses leaves the rest of that array to be
    staged piece by piece (``Issued``)."""

    def __init__(self, arrays, register: bool = True, lazy: bool | None = None):
        self.arrays = [a for a in arrays if a.nbytes]
        self.register = register and REGISTER
        self.lazy = LAZY_REGISTER if lazy is None else lazy
        self.done = []  # start addresses of our registrations
        self.spans: list[_Span] = []
        self._keys = []
        self.ok = False
        self.stats = {"registrations": 0, "register_ms": 0.0, "staged_bytes": 0}

    def _reg(self, p0: int, p1: int) -> bool:
        t0 = time.perf_counter()
        hip = _hip()
        rc = hip.hipHostRegister(ctypes.c_void_p(p0), ctypes.c_size_t(p1 - p0), ctypes.c_uint(0))
        self.stats["register_ms"] += 1e3 * (time.perf_counter() - t0)
        if rc != 0:
            hip.hipGetLastError()  # clear the refused call's error state
            return False
        self.done.append(p0)
        self.stats["registrations"] += 1
        return True

    def __enter__(self):
        for a in self.arrays:
            if RESULTS.contains(a):  # one of our pooled results: registered already
                continue
            if not self.register:
                self.__exit__(None, None, None)
                return self
            p0, p1 = a.ctypes.data, a.ctypes.data + a.nbytes
            if self.lazy and a.nbytes >= LAZY_MIN_BYTES:
                self.spans.append(_Span(p0, p1))
            elif not self._reg(p0, p1):
                self.__exit__(None, None, None)
                return self
        self.spans.sort(key=lambda sp: sp.start)
        self._keys = [sp.start for sp in self.spans]
        self.ok = True
        return self

    def split(self, a: np.ndarray) -> list[tuple[int, int, bool]]:
        """Byte ranges (b0, b1, registered) covering contiguous piece ``a`` of
        one of the arrays, each inside one registration, registering what
        the piece needs first.  Pieces of an array come in address order.
        A range the driver refused (and everything after it in that array)
        comes back unregistered: ``Issued`` stages it."""
        p0, p1 = a.ctypes.data, a.ctypes.data + a.nbytes
        i = bisect.bisect_right(self._keys, p0) - 1
        if i < 0 or not p1 <= self.spans[i].end:
            return [(0, a.nbytes, True)]  # registered whole on entry, or pooled
        sp = self.spans[i]
        if sp.reg_end < p1 and not sp.refused:
            grown = sp.base + LAZY_GROWTH * (sp.reg_end - sp.base)
            new = min(sp.cap, max(-(-p1 // PAGE) * PAGE, -(-grown // PAGE) * PAGE))
            if self._reg(sp.reg_end, new):
                if sp.reg_end > sp.base:
                    sp.joins.append(sp.reg_end)
                sp.reg_end = new
            else:
                sp.refused = True
        out, cur = [], p0
        for c in sp.joins:
            if cur < c < p1:
                out.append((cur - p0, c - p0, True))
                cur = c
        if p1 <= sp.reg_end:
            out.append((cur - p0, p1 - p0, True))
        else:
            if cur < sp.reg_end:
                out.append((cur - p0, sp.reg_end - p0, True))
                cur = sp.reg_end
            out.append((cur - p0, p1 - p0, False))
            self.stats["staged_bytes"] += p1 - cur
        return out

    def __exit__(self, *exc):
        hip = _hip()
        while self.done:
            hip.hipHostUnregister(ctypes.c_void_p(self.done.pop()))
        self.spans, self._keys = [], []
        return False


_HIP = None


def _hip():
    global _HIP
    if _HIP is None:
        _HIP = ctypes.CDLL("libamdhip64.so")
    return _HIP


_STREAMS: dict = {}


def streams(dev):
    """(h2d, compute, d2h) torch streams of ``dev``, made once per device."""
    import torch

    key = str(dev)
    s = _STREAMS.get(key)
    if s is None:
        s = tuple(torch.cuda.Stream(dev) for _ in range(3))
        _STREAMS[key] = s
    return s


def host_layers(xs, dtype) -> list[np.ndarray]:
    """Each layer as a flat ``dtype`` array: the caller's own memory when it
    already is a C-contiguous one (staged from in place), else a converted
    copy."""
    out = []
    for a in xs:
        a = np.asarray(a)
        if a.dtype != dtype or not a.flags.c_contiguous:
            a = np.ascontiguousarray(a, dtype=dtype)
        out.append(a.reshape(-1))
    return out


def pieces(layers: list[np.ndarray], lo: int, hi: int) -> list[tuple[np.ndarray, int]]:
    """The layers' elements [lo, hi) of their concatenation as (host piece,
    offset from lo) pairs, for ``Feeder``."""
    out, off = [], 0
    for a in layers:
        end = off + a.size
        a0, a1 = max(lo, off), min(hi, end)
        if a0 < a1:
            out.append((a[a0 - off:a1 - off], a0 - lo))
        off = end
        if off >= hi:
            break
    return out


class Phases:
    """Phase timer of one pipelined call (printed under SFL_HOSTPIPE_TRACE)."""

    def __init__(self, what: str):
        self.what, self.t0, self.marks = what, time.perf_counter(), []

    def mark(self, name: str) -> None:
        if TRACE:
            self.marks.append((name, time.perf_counter()))

    def note(self, **kw) -> None:
        if TRACE:
            self.marks.append((" ".join(f"{k}={v:.2f}" if isinstance(v, float) else f"{k}={v}"
                                        for k, v in kw.items()), None))

    def done(self) -> None:
        if TRACE:
            t, parts = self.t0, []
            for name, tm in self.marks:
                if tm is None:
                    parts.append(f"[{name}]")
                    continue
                parts.append(f"{name} {1e3 * (tm - t):.2f}")
                t = tm
            print(f"[hostpipe] {self.what}: " + ", ".join(parts) + f" | total {1e3 * (t - self.t0):.2f} ms",
                  file=sys.stderr, flush=True)
