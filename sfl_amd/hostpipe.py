"""Host-array <-> GPU pipelining for the drop-in's large payloads.

A party's ``mask_payload`` and the server's ``sum_decode`` start and end in
host memory (numpy arrays a secretflow PYU hands over and ships on).  For a
large payload the time is the PCIe copies (``tools/pcie_paths.py`` on
MI355X: ~57 GB/s each way, ~79 GB/s both ways at once; a pageable copy
runs at the same rate but blocks the host until it is done), not the
kernels (a 100M-element party mask is ~0.5 ms of device time).  So:

* the caller's host arrays are copied from where they are (no staging copy
  into pinned memory), by a helper thread (``Feeder``): a pageable copy
  runs at the pinned rate but blocks the thread that issues it;
* the result goes into a recycled registered buffer (``ResultPool``: free
  once the caller dropped every array viewing it), so the D2H is async DMA
  into pages that are in; on a miss, into a fresh array whose chunks a
  thread pool faults in ahead of the copies (first touch of fresh memory is
  the cost), chunk j's D2H a pageable copy as soon as its pages are in;
* the element range is cut into chunks; chunk j's H2D (the feeder's
  stream), its kernels (a second) and its D2H (a third, from the calling
  thread) overlap with chunk j+1's, the streams ordered by events.

Nothing here computes: the kernels are the library's (``sa_mask``,
``sa_xor_u64``, ``sa_sum_u64``, ``sa_decode``).  Used by
``security/aggregation/party.py``.
"""

from __future__ import annotations

import ctypes
import os
import sys
import threading
import time
from concurrent.futures import ThreadPoolExecutor

import numpy as np

_POOL = None
# SFL_HOSTPIPE_TRACE=1: every pipelined call prints its phase times to stderr
TRACE = os.environ.get("SFL_HOSTPIPE_TRACE") == "1"
_POOL_LOCK = threading.Lock()
TOUCH_THREADS = 8
PAGE = 4096


def _pool() -> ThreadPoolExecutor:
    global _POOL
    with _POOL_LOCK:
        if _POOL is None:
            _POOL = ThreadPoolExecutor(TOUCH_THREADS, thread_name_prefix="sfl_sa_touch")
    return _POOL


def chunk_bounds(n: int, target: int = 8, lo_elems: int = 1 << 20, hi_elems: int = 1 << 24,
                 align: int = 1024) -> list[tuple[int, int]]:
    """[0, n) in about ``target`` chunks of lo_elems..hi_elems elements, each
    start a multiple of ``align`` (16-byte aligned device slices)."""
    if n <= 0:
        return []
    step = min(max(-(-n // target), lo_elems), hi_elems)
    step = -(-step // align) * align
    return [(lo, min(n, lo + step)) for lo in range(0, n, step)]


class FreshOutput:
    """A host result of ``n`` elements that the device fills chunk by chunk:
    a recycled registered buffer from ``RESULTS`` when one is free (no
    faults, async copies), else ``np.empty`` memory (numpy advises huge pages for large
    allocations: its first touch runs at ~27 GB/s on one thread, against
    ~8 GB/s for a plain anonymous mmap -- tools/touch_probe.py), faulted in
    by the thread pool in chunk order from construction on; ``ready(j)``
    waits for chunk j's pages.  The D2H into a ready chunk is a pageable
    copy (55 GB/s into touched pages, like a registered one): registering a
    fresh result costs more than it saves (hipHostRegister takes the mm lock
    and stalls the faulting threads).  ``array`` is the caller's result."""

    def __init__(self, n: int, dtype, bounds):
        dtype = np.dtype(dtype)
        self.bounds = bounds
        self.stats = {"wait_ms": 0.0, "pooled": False}
        self._futs = [[] for _ in bounds]
        owner = RESULTS.take(n * dtype.itemsize)
        if owner is not None:  # a recycled, registered buffer: no faults, async DMA
            self.array = owner[:n * dtype.itemsize].view(dtype)
            self.stats["pooled"] = True
            return
        self.array = np.empty(n, dtype=dtype)
        self._b = self.array.view(np.uint8).reshape(-1)
        isz = dtype.itemsize
        pool = _pool()
        self._futs = []
        for lo, hi in bounds:
            b0, b1 = lo * isz, hi * isz
            step = max(PAGE, -(-(b1 - b0) // TOUCH_THREADS) // PAGE * PAGE)
            self._futs.append([pool.submit(self._touch, a, min(b1, a + step)) for a in range(b0, b1, step)])

    def _touch(self, a: int, b: int) -> None:
        self._b[a:b:PAGE] = 0
        self._b[b - 1] = 0  # the last page of the range

    def ready(self, j: int) -> np.ndarray:
        """Chunk j's elements, faulted in."""
        t0 = time.perf_counter()
        for f in self._futs[j]:
            f.result()
        self.stats["wait_ms"] += 1e3 * (time.perf_counter() - t0)
        lo, hi = self.bounds[j]
        return self.array[lo:hi]

    def close(self) -> None:
        for f in (f for fs in self._futs for f in fs):
            f.result()  # no toucher may outlive the call


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
            step = -(-nbytes // TOUCH_THREADS) // PAGE * PAGE + PAGE

            def touch(lo):
                owner[lo:lo + step:PAGE] = 0

            list(_pool().map(touch, range(0, nbytes, step)))
            hip = _hip()
            if hip.hipHostRegister(ctypes.c_void_p(owner.ctypes.data), ctypes.c_size_t(nbytes), ctypes.c_uint(0)):
                hip.hipGetLastError()
                return None
            self.bufs.append(owner)
            return owner

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
    """The H2D side of a pipelined call, on a helper thread: ``jobs[j]()``
    issues chunk j's host-to-device copies on ``stream`` (the caller's own
    pageable arrays: a pageable copy runs at the pinned rate but blocks the
    thread that issues it -- tools/pcie_paths.py -- so it gets a thread of
    its own; registering the arrays instead costs up to 8 ms per 800 MB and
    stalls page faults elsewhere).  ``ready(j)`` returns the device event
    that chunk j's copies complete at, once they are issued."""

    def __init__(self, stream, jobs):
        self.stream, self.jobs = stream, jobs
        self.flags = [threading.Event() for _ in jobs]
        self.events = [None] * len(jobs)
        self.error = None
        self.thread = threading.Thread(target=self._run, name="sfl_sa_h2d", daemon=True)
        self.thread.start()

    def _run(self) -> None:
        import torch

        try:
            with torch.cuda.device(self.stream.device), torch.cuda.stream(self.stream):
                for j, job in enumerate(self.jobs):
                    job()
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
    """``Feeder``'s interface for inputs that need no thread (registered):
    every chunk's copies issued on ``stream`` at construction, from the
    calling thread."""

    def __init__(self, stream, jobs):
        import torch

        self.events = []
        with torch.cuda.stream(stream):
            for job in jobs:
                job()
                e = torch.cuda.Event()
                e.record(stream)
                self.events.append(e)

    def ready(self, j: int):
        return self.events[j]

    def join(self, check: bool = True) -> None:
        pass


class Pinned:
    """hipHostRegister the caller's input arrays for a ``with`` block, so
    their H2D copies are true async DMA issued from the calling thread
    (the per-party mask step: its pageable H2D and pageable D2H would
    otherwise take turns -- 22.6 against 19.0 ms for 100M floats).  ``ok`` is
    False when the driver refuses any of them (then nothing stays registered
    and the caller feeds pageable copies from a thread).  Unregistered on
    exit, whatever happened."""

    def __init__(self, arrays):
        self.arrays = [a for a in arrays if a.nbytes]
        self.done = []
        self.ok = False

    def __enter__(self):
        hip = _hip()
        for a in self.arrays:
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
    """Each layer as a flat C-contiguous ``dtype`` array: the caller's own
    memory when it already is one (copied from in place), else a converted
    copy."""
    out = []
    for a in xs:
        a = np.asarray(a)
        if a.dtype != dtype or not a.flags.c_contiguous:
            a = np.ascontiguousarray(a, dtype=dtype)
        out.append(a.reshape(-1))
    return out


def copy_pieces(dst, layers: list[np.ndarray], lo: int, hi: int) -> None:
    """dst[lo:hi] (a device tensor, the layers' concatenation) <- the layers'
    elements [lo, hi), one copy per overlapping layer on the current stream."""
    import warnings

    import torch

    off = 0
    for a in layers:
        end = off + a.size
        a0, a1 = max(lo, off), min(hi, end)
        if a0 < a1:
            with warnings.catch_warnings():  # a read-only caller array is only read here
                warnings.filterwarnings("ignore", message="The given NumPy array is not writable")
                src = torch.from_numpy(a[a0 - off:a1 - off])
            dst[a0:a1].copy_(src, non_blocking=True)
        off = end
        if off >= hi:
            break


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
