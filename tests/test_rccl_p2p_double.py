"""The `direct` exchange's and the float64 gather's send/recv slot arithmetic
with 2..8 ranks, on the CPU.

RCCL refuses two ranks on one GPU and no multi-GPU box is ours, so
``sa_comm_alltoall_u64`` and ``sa_comm_gather_f64`` (sfl_amd/csrc/sa_rccl.cpp,
the product source, compiled as it is) are linked against a test double of
RCCL's point-to-point subset (tests/c_abi/rccl_p2p_double.cpp: ranks are
threads, groups matched per (source, destination) at ncclGroupEnd, an
unmatched or mis-sized send/recv fails).  Each rank's receive slot p must hold
rank p's shard of this rank, its own slot untouched; every root's gather
holds the ranks' shards in rank order; ``sa_comm_info`` reports W ranks and the
rank's own index and device.  What this cannot show is RCCL's own
behaviour on xGMI (the driver's 8-GPU run); it pins this file's indexing."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HIPCC = "/opt/rocm/bin/hipcc"


@pytest.fixture(scope="module")
def double_bin(tmp_path_factory):
    if not os.path.exists(HIPCC) or shutil.which("g++") is None:
        pytest.skip("needs hipcc and g++")
    d = tmp_path_factory.mktemp("rccl_double")
    flags = ["-fPIC", "-O1", "-std=c++17", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include"]
    objs = []
    for src in (os.path.join(ROOT, "sfl_amd", "csrc", "sa_rccl.cpp"),
                os.path.join(ROOT, "tests", "c_abi", "rccl_p2p_double.cpp")):
        o = str(d / (os.path.basename(src) + ".o"))
        subprocess.run([HIPCC, *flags, "-c", src, "-o", o], check=True)
        objs.append(o)
    exe = str(d / "rccl_double")
    subprocess.run(["g++", *objs, "-o", exe, "-lpthread"], check=True)
    return exe


@pytest.mark.parametrize("world", [1, 2, 3, 4, 8])
@pytest.mark.parametrize("count", [1, 1001])
def test_direct_exchange_and_gather_slots(double_bin, world, count):
    r = subprocess.run([double_bin, str(world), str(count)], capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    assert r.stdout.strip() == f"ok world={world} count={count}"
