"""Every sa_comm_* collective with REAL multi-rank RCCL on the box's one GPU
(tools/rccl_hostid_probe.py): a distinct NCCL_HOSTID per rank makes each rank
its own RCCL node, connected through RCCL's socket transport on lo -- the
duplicate-GPU check compares (host hash, bus id).  reduce-scatter in place
(with uint64 wrap-around), all-to-all (own slot untouched), float64 gather,
reduce to a root, all-reduce: checked against the expected values on every
rank."""
import json
import os
import subprocess
import sys

import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.parametrize("world", [3, 8])
def test_every_collective_between_real_rccl_ranks(world):
    if torch.cuda.device_count() == 0:  # asked without initialising HIP in this process
        pytest.skip("no GPU")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "rccl_hostid_probe.py"), "--world", str(world)],
                       capture_output=True, text=True, timeout=200, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    dec, res, i = json.JSONDecoder(), [], r.stdout.find("PROBE ")
    while i >= 0:  # every "PROBE {...}" record, wherever the ranks' lines fell
        obj, end = dec.raw_decode(r.stdout, i + len("PROBE "))
        res.append(obj)
        i = r.stdout.find("PROBE ", end)
    assert sorted(x["rank"] for x in res) == list(range(world)), r.stdout
    for x in res:
        assert "error" not in x, x
        keys = ["reduce_scatter", "reduce_scatter_wraps", "alltoall", "allreduce"] + (
            ["gather", "reduce"] if x["rank"] == 0 else [])
        assert all(x[k] is True for k in keys), x
