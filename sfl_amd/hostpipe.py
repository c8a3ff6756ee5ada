"""Host-array <-> GPU pipelining for the drop-in's large payloads.

A party's ``mask_payload`` and the server's ``sum_decode`` start and end in
host memory (numpy arrays a secretflow PYU hands over and ships on).  For a
large payload the time is the PCIe copies (``tools/pcie_paths.py`` on
MI355X: ~57 GB/s each way, ~79 GB/s both ways at once; a pageable copy
runs at the same rate but blocks the host until it is done), not the
kernels (a 100M-element party mask is ~0.5 ms of device time).  So:

* the caller's host arrays are HIP-registered in place for the call
  (``hipHostRegister``: no staging copy through a pinned bounce buffer);
* the result goes into a FRESH host array (the caller keeps it): anonymous
  memory whose chunks are faulted in by a thread pool (first touch of fresh
  memory runs at ~14 GB/s on one thread) and registered chunk by chunk, so
  chunk j's D2H starts while later chunks are still being faulted in;
* the element range is cut into chunks; chunk j's H2D (one stream), its
  kernels (a second) and its D2H (a third) overlap with chunk j+1's, the
  streams ordered by events.

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

_HIP = None
_POOL = None
# SFL_HOSTPIPE_TRACE=1: every pipelined call prints its phase times to stderr
TRACE = os.environ.get("SFL_HOSTPIPE_TRACE") == "1"
_POOL_LOCK = threading.Lock()
TOUCH_THREADS = 8
PAGE = 4096


def _hip():
    global _HIP
    if _HIP is None:
        _HIP = ctypes.CDLL("libamdhip64.so")
    return _HIP


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
    """A fresh host result of ``n`` elements that the device fills chunk by
    chunk: page-aligned anonymous memory (``mmap``) whose chunks are faulted
    in by the thread pool, in chunk order, from construction on; ``ready(j)``
    waits for chunk j's pages and HIP-registers exactly them, so chunk j's
    D2H can start while later chunks are still being faulted in (first touch
    of fresh memory is the cost: ~14 GB/s on one thread).  ``array`` is the
    caller's result (it keeps the mapping alive); ``close()`` unregisters.
    A chunk whose registration is refused is copied pageable (correct,
    synchronous)."""

    def __init__(self, n: int, dtype, bounds):
        import mmap

        self.dtype = np.dtype(dtype)
        nbytes = n * self.dtype.itemsize
        self.size = max(PAGE, -(-nbytes // PAGE) * PAGE)
        # private anonymous pages (Python's default for fd -1 is MAP_SHARED:
        # shmem-backed pages, slower to fault and to register)
        self._mm = mmap.mmap(-1, self.size, flags=mmap.MAP_PRIVATE | mmap.MAP_ANONYMOUS)
        self.array = np.frombuffer(self._mm, dtype=self.dtype, count=n)
        self._b = np.frombuffer(self._mm, dtype=np.uint8)
        self.base = self.array.ctypes.data
        self.bounds = bounds
        self.registered = []
        self.stats = {"wait_ms": 0.0, "register_ms": 0.0, "refused": 0}
        pool = _pool()
        self._futs = []
        for lo, hi in bounds:
            b0, b1 = self._span(lo, hi)
            step = max(PAGE, -(-(b1 - b0) // TOUCH_THREADS) // PAGE * PAGE)
            self._futs.append([pool.submit(self._touch, a, min(b1, a + step)) for a in range(b0, b1, step)])

    def _span(self, lo: int, hi: int) -> tuple[int, int]:
        """Byte range of elements [lo, hi), widened to whole pages (chunk
        starts are page-aligned: chunk_bounds aligns them to 1024 elements)."""
        isz = self.dtype.itemsize
        return (lo * isz) // PAGE * PAGE, min(self.size, -(-(hi * isz) // PAGE) * PAGE)

    def _touch(self, a: int, b: int) -> None:
        self._b[a:b:PAGE] = 0

    def ready(self, j: int) -> np.ndarray:
        """Chunk j's elements, faulted in and (when the driver accepts it)
        registered."""
        t0 = time.perf_counter()
        for f in self._futs[j]:
            f.result()
        t1 = time.perf_counter()
        lo, hi = self.bounds[j]
        b0, b1 = self._span(lo, hi)
        if b1 > b0:
            hip = _hip()
            rc = hip.hipHostRegister(ctypes.c_void_p(self.base + b0), ctypes.c_size_t(b1 - b0), ctypes.c_uint(0))
            if rc == 0:
                self.registered.append(self.base + b0)
            else:
                hip.hipGetLastError()
                self.stats["refused"] += 1
        self.stats["wait_ms"] += 1e3 * (t1 - t0)
        self.stats["register_ms"] += 1e3 * (time.perf_counter() - t1)
        return self.array[lo:hi]

    def close(self) -> None:
        for f in (f for fs in self._futs for f in fs):
            f.result()  # no toucher may outlive the call
        hip = _hip()
        while self.registered:
            hip.hipHostUnregister(ctypes.c_void_p(self.registered.pop()))


class Registered:
    """hipHostRegister the given C-contiguous numpy arrays for a ``with``
    block, so device copies run as true async DMA from / into them;
    unregistered on exit, whatever happened.  ``usable[i]`` is the array to
    copy through: ``arrays[i]`` itself, or -- when its pages cannot be
    registered (already registered by someone else, or sharing a page with
    memory that is) -- a page-locked copy (an input) or a page-locked
    stand-in whose contents ``__exit__`` copies back (an output,
    ``outputs``).  Empty arrays are passed through."""

    def __init__(self, arrays, outputs=()):
        self.arrays = list(arrays)
        self.outputs = {id(a) for a in outputs}  # stand-ins of these are copied back on exit
        self.done, self.back = [], []
        self.usable = []

    def __enter__(self):
        import torch

        hip = _hip()
        try:
            for a in self.arrays:
                if not a.flags.c_contiguous:
                    raise ValueError("only C-contiguous arrays can be registered")
                if a.nbytes == 0:
                    self.usable.append(a)
                    continue
                rc = hip.hipHostRegister(ctypes.c_void_p(a.ctypes.data), ctypes.c_size_t(a.nbytes),
                                         ctypes.c_uint(0))
                if rc == 0:
                    self.done.append(a)
                    self.usable.append(a)
                    continue
                hip.hipGetLastError()  # clear the refused call's error state
                stand = torch.empty(a.nbytes, dtype=torch.uint8, pin_memory=True).numpy().view(a.dtype)
                if id(a) in self.outputs:
                    self.back.append((a, stand))
                else:
                    np.copyto(stand, a)
                self.usable.append(stand)
        except BaseException:
            self.__exit__(None, None, None)
            raise
        return self

    def __exit__(self, exc_type, *exc):
        hip = _hip()
        while self.done:
            a = self.done.pop()
            hip.hipHostUnregister(ctypes.c_void_p(a.ctypes.data))
        if exc_type is None:
            for a, stand in self.back:
                np.copyto(a, stand)
        self.back = []
        return False


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
    memory when it already is one (registered in place), else a converted
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
    elements [lo, hi), one async copy per overlapping layer on the current
    stream (the layers are registered)."""
    import torch

    off = 0
    for a in layers:
        end = off + a.size
        a0, a1 = max(lo, off), min(hi, end)
        if a0 < a1:
            dst[a0:a1].copy_(torch.from_numpy(a[a0 - off:a1 - off]), non_blocking=True)
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
