"""Host-array <-> GPU pipelining for the drop-in's large payloads.

A party's ``mask_payload`` and the server's ``sum_decode`` start and end in
host memory (numpy arrays a secretflow PYU hands over and ships on).  For a
large payload the time is the PCIe copies (``tools/pcie_paths.py`` on
MI355X: ~57 GB/s each way, ~79 GB/s both ways at once), not the kernels (a
100M-element party mask is ~0.5 ms of device time).  So:

* the element range is cut into chunks; chunk j's H2D, its kernels and its
  D2H run on three streams ordered by events, overlapping chunk j+1's;
* every DMA touches page-locked memory only: the caller's arrays are
  staged through pinned slots (torch's caching host allocator) by a feeder
  thread whose memcpy runs on a thread pool (75-97 GB/s on 8-16 threads,
  above the PCIe rate, tools/pcie_paths.py); the caller's memory is never registered and no copy is
  pageable (pageable D2H copies into fresh arrays beside registered
  memory failed now and then with hipErrorInvalidValue, once aborting in
  the next synchronise);
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


def chunk_bounds(n: int, target: int = 8, lo_elems: int = 1 << 20, hi_elems: int = 1 << 24,
                 align: int = 1024) -> list[tuple[int, int]]:
    """[0, n) in about ``target`` chunks of lo_elems..hi_elems elements, each
    start a multiple of ``align`` (16-byte aligned device slices)."""
    if n <= 0:
        return []
    step = min(max(-(-n // target), lo_elems), hi_elems)
    step = -(-step // align) * align
    return [(lo, min(n, lo + step)) for lo in range(0, n, step)]


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
    overlapped them."""

    LOOKAHEAD = 1

    def __init__(self, stream, chunks):
        self.stream, self.chunks = stream, chunks
        self.events = []

    def _issue(self, j: int) -> None:
        import torch

        with torch.cuda.stream(self.stream):
            for dst, pcs in self.chunks[j]:
                for a, off in pcs:
                    dst[off:off + a.size].copy_(_tensor(a), non_blocking=True)
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


class Pinned:
    """hipHostRegister a party's input layers for a ``with`` block, so their
    H2D is async DMA issued at once (``Issued``) instead of staged by the
    feeder: the party's 400 MB in then overlaps its 800 MB out completely
    (16.3 against ~27 ms for 100M floats).  Only our own copies touch these
    pages while they are registered, and none of them is pageable.  Arrays
    inside a pooled result (``RESULTS``: e.g. the masked vectors the server
    receives from parties in the same process) are registered already and
    taken as they are; with ``register=False`` nothing else is registered
    (``ok`` then says whether every array was pooled).  ``ok`` is False when
    the driver refuses any array (already registered elsewhere, or sharing a
    page with registered memory): nothing stays registered and the caller
    stages through the feeder.  Unregistered on exit."""

    def __init__(self, arrays, register: bool = True):
        self.arrays = [a for a in arrays if a.nbytes]
        self.register = register
        self.done = []
        self.ok = False

    def __enter__(self):
        hip = _hip()
        for a in self.arrays:
            if RESULTS.contains(a):  # one of our pooled results: registered already
                continue
            if not self.register:
                self.__exit__(None, None, None)
                return self
            rc = hip.hipHostRegister(ctypes.c_void_p(a.ctypes.data), ctypes.c_size_t(a.nbytes), ctypes.c_uint(0))
            if rc != 0:
                hip.hipGetLastError()  # clear the refused call's error state
                self.__exit__(None, None, None)
                return self
            self.done.append(a)
        self.ok = True
        return self

    def __exit__(self, *exc):
        hip = _hip()
        while self.done:
            hip.hipHostUnregister(ctypes.c_void_p(self.done.pop().ctypes.data))
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
