"""The drop-in boundary on CPU: libsfl_sa.so loads, exports every symbol
include/sfl_sa.h declares, its host-side setup math equals numpy, and the
product package never reaches for the oracle or a CPU fallback."""
import os
import re

import numpy as np
import pytest

from oracle import secagg as o

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _declared():
    hdr = open(os.path.join(ROOT, "include", "sfl_sa.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:int|const char\*)\s+(sa_\w+)\s*\(", hdr, flags=re.M)))


def test_library_exports_every_declared_symbol():
    from sfl_amd import _lib as L

    lib = L.lib()
    declared = _declared()
    assert len(declared) >= 15
    for name in declared:
        assert hasattr(lib, name), name
    assert set(declared) == set(L.EXPORTED)
    assert lib.sa_abi_version() == 3


def test_library_is_built_for_gfx950():
    import subprocess

    so = os.path.join(ROOT, "sfl_amd", "lib", "libsfl_sa.so")
    out = subprocess.run(["/opt/rocm/bin/roc-obj-ls", so], capture_output=True, text=True)
    if out.returncode != 0:
        pytest.skip("roc-obj-ls unavailable")
    assert "gfx950" in out.stdout


@pytest.mark.parametrize("seed", [0, 1, 42, o.pair_seed(0, 7), 2**63 + 11, 2**64, 2**127 + 5, 3**100])
def test_seeding_matches_numpy(seed):
    from sfl_amd import _lib as L

    g = L.pcg64_from_seed(seed)
    assert g.pair() == o.pcg64_state(seed)


@pytest.mark.parametrize("delta", [0, 1, 3, 1023, 2**32 + 7, 2**70 + 1])
def test_advance_and_host_draws_match_numpy(delta):
    from sfl_amd import _lib as L

    seed = o.pair_seed(2, 3)
    g = L.pcg64_advance(L.pcg64_from_seed(seed), delta)
    bg = np.random.PCG64(seed)
    bg.advance(delta)
    assert g.state.value() == bg.state["state"]["state"]
    assert np.array_equal(L.pcg64_raw_host(g, 6), bg.random_raw(6))


def test_advance_many_equals_one_by_one():
    """sa_pcg64_advance_many (one call for a round's streams) == per-stream
    sa_pcg64_advance == numpy's PCG64.advance, including delta 0 and in-place
    output."""
    from sfl_amd import _lib as L

    gens = [L.pcg64_from_seed(7 + i) for i in range(6)]
    deltas = [0, 1, 2, 1000003, 2**40 + 7, 2**64 - 1]
    many = [g.pair() for g in L.pcg64_advance_many(gens, deltas)]
    assert many == [L.pcg64_advance(g, d).pair() for g, d in zip(gens, deltas)]
    bg = np.random.PCG64(9)
    st = bg.state["state"]
    bg.advance(12345)
    g = L.pcg64_advance_many([L.PCG64.of(st["state"], st["inc"])], [12345])[0]
    assert g.pair() == (bg.state["state"]["state"], bg.state["state"]["inc"])
    assert L.pcg64_advance_many([], []) == []


def test_errors_cross_the_abi_as_codes():
    import ctypes as C

    from sfl_amd import _lib as L

    lib = L.lib()
    rc = lib.sa_mask(None, 0, 0, 10, 1.0, None, 18, None, 0, None, None, None, None, None)
    assert rc == L.SA_ERR_ARG
    assert b"bad arguments" in lib.sa_last_error()
    rc = lib.sa_sum_u64(None, 0, 10, None, None)
    assert rc == L.SA_ERR_ARG
    with pytest.raises(L.SALibraryError):
        L.check(rc, "sa_sum_u64")
    arr = (C.c_uint32 * 1)(5)
    assert lib.sa_pcg64_from_seed(arr, -1, None) == L.SA_ERR_ARG


def test_every_entry_point_validates_before_touching_the_gpu():
    """Each export refuses bad arguments with SA_ERR_ARG and a message,
    before any HIP call (so this runs on a machine without a GPU); the
    reference's equivalent is a Python assert with a message
    (sparse_plain_aggregator.py:85).  n == 0 with valid sizes is a no-op."""
    from sfl_amd import _lib as L

    lib = L.lib()
    calls = {
        "sa_fused_clients": lambda: lib.sa_fused_clients(None, 0, 0, 10, 18, None, None, None, 0, None, 0, None,
                                                         None, None),
        "sa_decode": lambda: lib.sa_decode(None, 10, 63, 1.0, None, None, None),
        "sa_fused_bipartite": lambda: lib.sa_fused_bipartite(None, 0, 10, 18, None, None, None, 0, None, None),
        "sa_fused_clients_host_f32": lambda: lib.sa_fused_clients_host_f32(None, None, 2, 10, 18, None, None, 1.0,
                                                                           None, None, None, None, None, None),
        "sa_clients_host": lambda: lib.sa_clients_host(None, 2, 2, None, 2, 10, 18, None, 1.0, None, None, None,
                                                       None, None, None),
        "sa_mask_host": lambda: lib.sa_mask_host(None, 0, 0, 10, 1.0, 18, None, 0, None, None, None, None, None),
        "sa_sum_decode_host": lambda: lib.sa_sum_decode_host(None, 2, 10, 18, 1.0, None, None, None, None, None),
        "sa_sum_f64": lambda: lib.sa_sum_f64(None, 0, 10, None, None),
        "sa_pcg64_find_zero": lambda: lib.sa_pcg64_find_zero(None, 1, 10, None, None),
        "sa_stream_shift": lambda: lib.sa_stream_shift(None, 10, None, 1, 0, 1, None),
        "sa_xor_u64": lambda: lib.sa_xor_u64(None, 10, None, None),
        "sa_sumsq_f32": lambda: lib.sa_sumsq_f32(None, 10, None, None, 0, None),
        "sa_dp_perturb_f32": lambda: lib.sa_dp_perturb_f32(None, 10, None, None, None),
        "sa_mask_dp": lambda: lib.sa_mask_dp(None, 10, 1.0, 18, None, 0, None, None, None, None, None, None),
        "sa_mask": lambda: lib.sa_mask(None, 0, 0, 10, 1.0, None, 63, None, 0, None, None, None, None, None),
        "sa_comm_unique_id": lambda: lib.sa_comm_unique_id(None, 0),
        "sa_comm_init": lambda: lib.sa_comm_init(None, None, 0, 0, 0),
        "sa_comm_reduce_u64": lambda: lib.sa_comm_reduce_u64(None, None, None, 10, 0, None),
        "sa_comm_allreduce_u64": lambda: lib.sa_comm_allreduce_u64(None, None, None, 10, None),
        "sa_comm_reduce_scatter_u64": lambda: lib.sa_comm_reduce_scatter_u64(None, None, None, 10, None),
        "sa_comm_gather_f64": lambda: lib.sa_comm_gather_f64(None, None, None, 10, 0, None),
        "sa_comm_info": lambda: lib.sa_comm_info(None, None, None, None),
        "sa_pcg64_raw_host": lambda: lib.sa_pcg64_raw_host(None, None, 5),
        "sa_pcg64_advance_many": lambda: lib.sa_pcg64_advance_many(None, None, 3, None),
    }
    for name, call in calls.items():
        assert call() == L.SA_ERR_ARG, name
        assert lib.sa_last_error(), name
    assert lib.sa_mask(None, 0, 0, 0, 1.0, None, 18, None, 0, None, None, None, None, None) == L.SA_OK


def test_kernels_refuse_host_tensors():
    import torch

    from sfl_amd import kernels as K

    with pytest.raises(ValueError):
        K.sum_u64([torch.zeros(4, dtype=torch.int64)], torch.zeros(4, dtype=torch.int64))


def test_product_never_imports_the_oracle():
    pkg = os.path.join(ROOT, "sfl_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".hip", ".cpp", ".h")):
                src = open(os.path.join(dirpath, f)).read()
                assert not re.search(r"^\s*(from|import)\s+oracle", src, re.M), f
                assert "oracle/" not in src.replace("oracle/_ref", ""), f


def test_bench_runs_the_oracle_only_in_its_cpu_baseline_leg():
    """bench.py's measured path never touches the oracle: its only importer
    under bench.py / benchkit/ is the cpu_baseline leg (benchkit/baseline.py)."""
    srcs = {"bench.py": os.path.join(ROOT, "bench.py")}
    for f in os.listdir(os.path.join(ROOT, "benchkit")):
        if f.endswith(".py"):
            srcs[f"benchkit/{f}"] = os.path.join(ROOT, "benchkit", f)
    users = {k for k, p in srcs.items() if re.search(r"^\s*(from|import)\s+oracle", open(p).read(), re.M)}
    assert users == {"benchkit/baseline.py"}


def test_missing_library_fails_loudly(tmp_path, monkeypatch):
    import importlib

    import sfl_amd._lib as L

    monkeypatch.setenv("SFL_SA_LIB", str(tmp_path / "nope.so"))
    L2 = importlib.reload(L)
    try:
        with pytest.raises(L2.SALibraryError):
            L2.lib()
    finally:
        monkeypatch.delenv("SFL_SA_LIB")
        importlib.reload(L)


def test_every_entry_point_has_ctypes_signature():
    """ctypes converts Python floats only with declared argtypes: every
    exported entry point that takes arguments must have them."""
    from sfl_amd import _lib as L

    lib = L.lib()
    for name in L.EXPORTED:
        if name in ("sa_abi_version", "sa_last_error"):
            continue
        assert getattr(lib, name).argtypes, name


def test_tuning_builds_report_a_refused_abi_version(tmp_path):
    """SA_ABLATE (results WRONG) and SA_TIMING builds report ABI version
    1000 + 1, which sfl_amd._lib refuses unless a tuning tool opts in: a
    tuning library can never be loaded as the product."""
    import ctypes
    import subprocess

    from sfl_amd import _lib as L

    src = os.path.join(ROOT, "sfl_amd", "csrc", "sa_host.cpp")
    for define, want in (("", L.ABI_VERSION), ("-DSA_ABLATE=8", L.ABI_VERSION + L.TUNING_ABI_OFFSET),
                         ("-DSA_TIMING", L.ABI_VERSION + L.TUNING_ABI_OFFSET)):
        so = tmp_path / f"host{abs(hash(define))}.so"
        cmd = ["g++", "-std=c++17", "-shared", "-fPIC", "-O1", src, "-o", str(so)] + ([define] if define else [])
        subprocess.run(cmd, check=True, capture_output=True)
        assert ctypes.CDLL(str(so)).sa_abi_version() == want, define


def test_integration_table_cites_the_header_lines():
    """INTEGRATION.md's export table gives each entry point's line in
    include/sfl_sa.h: every ``name`` (line) pair must point at that
    declaration, and every declared entry point must be in the table."""
    hdr = open(os.path.join(ROOT, "include", "sfl_sa.h")).read().splitlines()
    table = [ln for ln in open(os.path.join(ROOT, "INTEGRATION.md")).read().splitlines()
             if ln.startswith("| `sa_")]
    cited = {}
    for row in table:
        for name, line in re.findall(r"`(sa_\w+)` \((\d+)\)", row.split("|")[1]):
            cited[name] = int(line)
    for name, line in cited.items():
        assert re.search(r"\b%s\(" % name, hdr[line - 1]), f"{name}: line {line} is {hdr[line - 1]!r}"
    declared = {m for ln in hdr for m in re.findall(r"^\w[\w\s\*]*\b(sa_\w+)\(", ln)}
    text = " ".join(r.split("|")[1] for r in table)
    missing = [d for d in declared if d not in text and "_" + d.split("_", 2)[-1] not in text]
    assert not missing, f"entry points missing from INTEGRATION.md's table: {missing}"


def test_ctypes_structs_match_the_header_layout(tmp_path):
    """The ctypes mirrors in sfl_amd/_lib.py have the C layout of
    include/sfl_sa.h (sizes and every field offset), compiled with gcc:
    ABI 3 changed sa_dp (a double clip), so a stale mirror would pass the
    wrong bytes silently."""
    import ctypes as C
    import shutil
    import subprocess

    from sfl_amd import _lib as L

    if shutil.which("gcc") is None:
        pytest.skip("no gcc")
    structs = {"sa_dp": (L.DP, ["sumsq", "sumsq_layer", "l2_norm_clip", "noise_std", "num_updates", "key",
                                "counter0"]),
               "sa_pcg64": (L.PCG64, ["state", "inc"]),
               "sa_mask_stream": (L.MaskStream, ["gen", "sign", "peer"]),
               "sa_local_client": (L.LocalClient, ["x", "weight", "masked_out"])}
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{os.path.join(ROOT, "include", "sfl_sa.h")}"',
             "int main(void) {"]
    for name, (_, fields) in structs.items():
        lines.append(f'  printf("{name} size %zu\\n", sizeof({name}));')
        for f in fields:
            lines.append(f'  printf("{name} {f} %zu\\n", offsetof({name}, {f}));')
    lines.append("  return 0;\n}")
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    r = subprocess.run(["gcc", "-std=c11", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", str(src), "-o", str(exe)],
                       capture_output=True, text=True)
    assert r.returncode == 0, r.stderr
    got = {}
    for ln in subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.splitlines():
        a, b, c = ln.split()
        got[(a, b)] = int(c)
    for name, (cls, fields) in structs.items():
        assert got[(name, "size")] == C.sizeof(cls), name
        for f in fields:
            assert got[(name, f)] == getattr(cls, f).offset, (name, f)
