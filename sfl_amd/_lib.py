"""ctypes binding of libsfl_sa.so (the C-ABI declared in include/sfl_sa.h).

The library is built in-tree by ``sfl_amd/csrc/Makefile`` (``__graft_entry__.build()``)
into ``sfl_amd/lib/libsfl_sa.so``.  There is no fallback: if the library is
missing or cannot be loaded, every hot-path call raises ``SALibraryError``.
"""

from __future__ import annotations

import ctypes as C
import os
import threading

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("SFL_SA_LIB", os.path.join(_HERE, "lib", "libsfl_sa.so"))

SA_OK = 0
SA_ERR_ARG = -1
SA_ERR_HIP = -2
SA_ERR_UNSUPPORTED = -3
SA_ERR_RCCL = -4

SA_F32, SA_F64, SA_I64 = 0, 1, 2
SA_FLAG_PRG_REJECT = 1
SA_UNIQUE_ID_BYTES = 128
SA_DP_PARTIALS = 1024
ABI_VERSION = 3  # include/sfl_sa.h SA_ABI_VERSION (3: the DP norm / clip follow numpy 1.23.5's float64 scalars)
TUNING_ABI_OFFSET = 1000  # sa_abi_version() of an SA_ABLATE / SA_TIMING build

# every symbol include/sfl_sa.h declares (checked by tests/test_boundary.py)
EXPORTED = (
    "sa_abi_version", "sa_last_error", "sa_pcg64_from_seed", "sa_pcg64_advance", "sa_pcg64_advance_many",
    "sa_pcg64_raw_host", "sa_mask", "sa_fused_clients", "sa_fused_clients_host_f32", "sa_clients_host", "sa_mask_host", "sa_sum_decode_host", "sa_fused_bipartite", "sa_set_masking_reserve", "sa_sum_u64", "sa_decode",
    "sa_sum_f64", "sa_comm_unique_id", "sa_comm_init", "sa_comm_reduce_u64",
    "sa_comm_allreduce_u64", "sa_comm_reduce_scatter_u64", "sa_comm_alltoall_u64", "sa_comm_gather_f64", "sa_comm_info", "sa_comm_destroy", "sa_sumsq_f32", "sa_dp_perturb_f32", "sa_mask_dp",
    "sa_pcg64_find_zero", "sa_stream_shift", "sa_xor_u64",
)


class SALibraryError(RuntimeError):
    """libsfl_sa.so is missing, failed to load, or a call returned an error."""


class U128(C.Structure):
    _fields_ = [("lo", C.c_uint64), ("hi", C.c_uint64)]

    @classmethod
    def of(cls, v: int) -> "U128":
        return cls(v & 0xFFFFFFFFFFFFFFFF, (v >> 64) & 0xFFFFFFFFFFFFFFFF)

    def value(self) -> int:
        return int(self.lo) | (int(self.hi) << 64)


class PCG64(C.Structure):
    _fields_ = [("state", U128), ("inc", U128)]

    @classmethod
    def of(cls, state: int, inc: int) -> "PCG64":
        return cls(U128.of(state), U128.of(inc))

    def pair(self) -> tuple[int, int]:
        return self.state.value(), self.inc.value()


class MaskStream(C.Structure):
    _fields_ = [("gen", PCG64), ("sign", C.c_int32), ("peer", C.c_int32)]


class LocalClient(C.Structure):
    _fields_ = [("x", C.c_void_p), ("weight", C.c_double), ("masked_out", C.c_void_p)]


class DP(C.Structure):
    """sa_dp: GaussianModelDP pre-step parameters."""
    _fields_ = [("sumsq", C.c_void_p), ("sumsq_layer", C.c_void_p), ("l2_norm_clip", C.c_double),
                ("noise_std", C.c_float), ("num_updates", C.c_float),
                ("key", C.c_uint64), ("counter0", C.c_uint64)]


_lock = threading.Lock()
_lib = None
_load_error: str | None = None


def _declare(lib):
    vp, u64, i32, dbl = C.c_void_p, C.c_uint64, C.c_int, C.c_double
    P = C.POINTER
    lib.sa_abi_version.restype = i32
    lib.sa_last_error.restype = C.c_char_p
    lib.sa_pcg64_from_seed.argtypes = [P(C.c_uint32), i32, P(PCG64)]
    lib.sa_pcg64_advance.argtypes = [P(PCG64), U128]
    lib.sa_pcg64_advance_many.argtypes = [P(PCG64), P(C.c_uint64), i32, P(PCG64)]
    lib.sa_pcg64_raw_host.argtypes = [P(PCG64), P(C.c_uint64), u64]
    lib.sa_mask.argtypes = [vp, i32, i32, u64, dbl, vp, i32, P(MaskStream), i32, vp, vp, vp, vp, vp]
    lib.sa_fused_clients.argtypes = [P(LocalClient), i32, i32, u64, i32, P(PCG64), P(C.c_int8),
                                     P(MaskStream), i32, vp, i32, vp, vp, vp]
    lib.sa_fused_clients_host_f32.argtypes = [P(C.c_void_p), P(C.c_double), i32, u64, i32, P(PCG64), P(C.c_int8),
                                              dbl, vp, vp, vp, vp, P(C.c_uint32), vp]
    lib.sa_clients_host.argtypes = [P(C.c_void_p), i32, i32, P(C.c_double), i32, u64, i32, P(MaskStream), dbl,
                                    vp, vp, vp, vp, P(C.c_uint32), vp]
    lib.sa_mask_host.argtypes = [vp, i32, i32, u64, dbl, i32, P(MaskStream), i32, vp, vp, vp, P(C.c_uint32), vp]
    lib.sa_sum_decode_host.argtypes = [P(C.c_void_p), i32, u64, i32, dbl, vp, vp, vp, vp, vp]
    lib.sa_fused_bipartite.argtypes = [P(LocalClient), i32, u64, i32, P(PCG64), P(C.c_int8), vp, i32, vp, vp]
    lib.sa_set_masking_reserve.argtypes = [i32]
    lib.sa_sum_u64.argtypes = [P(C.c_void_p), i32, u64, vp, vp]
    lib.sa_decode.argtypes = [vp, u64, i32, dbl, vp, vp, vp]
    lib.sa_sum_f64.argtypes = [P(C.c_void_p), i32, u64, vp, vp]
    lib.sa_comm_unique_id.argtypes = [vp, i32]
    lib.sa_comm_init.argtypes = [P(C.c_void_p), vp, i32, i32, i32]
    lib.sa_comm_reduce_u64.argtypes = [vp, vp, vp, u64, i32, vp]
    lib.sa_comm_allreduce_u64.argtypes = [vp, vp, vp, u64, vp]
    lib.sa_comm_reduce_scatter_u64.argtypes = [vp, vp, vp, u64, vp]
    lib.sa_comm_gather_f64.argtypes = [vp, vp, vp, u64, i32, vp]
    lib.sa_comm_alltoall_u64.argtypes = [vp, vp, vp, u64, vp]
    lib.sa_comm_info.argtypes = [vp, P(C.c_int), P(C.c_int), P(C.c_int)]
    lib.sa_comm_destroy.argtypes = [vp]
    lib.sa_sumsq_f32.argtypes = [vp, u64, vp, vp, i32, vp]
    lib.sa_dp_perturb_f32.argtypes = [vp, u64, P(DP), vp, vp]
    lib.sa_mask_dp.argtypes = [vp, u64, dbl, i32, P(MaskStream), i32, P(DP), vp, vp, vp, vp, vp]
    lib.sa_pcg64_find_zero.argtypes = [P(PCG64), i32, u64, vp, vp]
    lib.sa_stream_shift.argtypes = [vp, u64, P(PCG64), i32, u64, u64, vp]
    lib.sa_xor_u64.argtypes = [vp, u64, vp, vp]
    for name in EXPORTED:
        if name not in ("sa_last_error",):
            getattr(lib, name).restype = i32
    lib.sa_last_error.restype = C.c_char_p


def lib():
    """The loaded library; raises SALibraryError (never falls back)."""
    global _lib, _load_error
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is None:
            if not os.path.exists(LIB_PATH):
                _load_error = (f"{LIB_PATH} not found: build it with `python -c 'import "
                               f"__graft_entry__ as g; g.build()'` (make -C sfl_amd/csrc)")
                raise SALibraryError(_load_error)
            # torch first: its bundled libamdhip64.so.7 / librccl.so.1 then satisfy
            # our NEEDED entries by soname, so the process has ONE HIP runtime and
            # torch's hipStream_t handles are valid in our launches.
            import torch  # noqa: F401

            try:
                handle = C.CDLL(LIB_PATH, mode=C.RTLD_GLOBAL)
            except OSError as e:  # pragma: no cover - environment dependent
                _load_error = f"cannot load {LIB_PATH}: {e}"
                raise SALibraryError(_load_error) from e
            _declare(handle)
            ver = handle.sa_abi_version()
            if ver == ABI_VERSION + TUNING_ABI_OFFSET and os.environ.get("SFL_SA_ALLOW_TUNING_BUILD") == "1":
                pass  # tools/ timing a tuning variant on purpose (never the product)
            elif ver != ABI_VERSION:
                raise SALibraryError(
                    f"{LIB_PATH}: ABI version {ver}" + (" (a tuning build: SA_ABLATE / SA_TIMING; results of "
                                                        "ablation builds are wrong)" if ver > TUNING_ABI_OFFSET
                                                        else " mismatch"))
            _lib = handle
    return _lib


def check(rc: int, what: str) -> None:
    if rc != SA_OK:
        msg = lib().sa_last_error().decode(errors="replace")
        raise SALibraryError(f"{what} failed with code {rc}: {msg}")


# ---------------------------------------------------------------------------
# host-side generator setup (no GPU required)
# ---------------------------------------------------------------------------

def _int_words(seed: int) -> list[int]:
    if seed < 0:
        raise ValueError("seed must be non-negative")
    words = []
    while True:
        words.append(seed & 0xFFFFFFFF)
        seed >>= 32
        if seed == 0:
            break
    return words


def pcg64_from_seed(seed: int) -> PCG64:
    """numpy ``PCG64(seed)`` state, computed by the library (SeedSequence)."""
    w = _int_words(int(seed))
    arr = (C.c_uint32 * len(w))(*w)
    out = PCG64()
    check(lib().sa_pcg64_from_seed(arr, len(w), C.byref(out)), "sa_pcg64_from_seed")
    return out


def pcg64_advance(g: PCG64, delta: int) -> PCG64:
    out = PCG64(g.state, g.inc)
    check(lib().sa_pcg64_advance(C.byref(out), U128.of(int(delta))), "sa_pcg64_advance")
    return out


def pcg64_advance_many(gens, deltas) -> list:
    """[pcg64_advance(g, d) for g, d in zip(gens, deltas)] in one library call
    (deltas below 2^64)."""
    k = len(gens)
    if k == 0:
        return []
    arr = (PCG64 * k)(*gens)
    ds = (C.c_uint64 * k)(*[int(d) for d in deltas])
    check(lib().sa_pcg64_advance_many(arr, ds, k, arr), "sa_pcg64_advance_many")
    return list(arr)


def pcg64_raw_host(g: PCG64, n: int):
    import numpy as np

    out = np.empty(n, dtype=np.uint64)
    tmp = PCG64(g.state, g.inc)
    check(lib().sa_pcg64_raw_host(C.byref(tmp), out.ctypes.data_as(C.POINTER(C.c_uint64)), n),
          "sa_pcg64_raw_host")
    return out
