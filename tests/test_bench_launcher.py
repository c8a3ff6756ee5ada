"""bench.py's multi-GPU launch contract, rehearsed on the CPU (--dry-run: the
ranks join a gloo group instead of touching a GPU).

* ``python bench.py --gpus N`` with no outer torchrun starts N rank processes
  itself (one torch.distributed.run child) and exactly ONE JSON line comes
  back, from rank 0, carrying the CPU baseline the parent measured before
  any rank started;
* under an outer ``torch.distributed.run`` (the driver's form) every rank is
  a worker and rank 0 measures the CPU baseline itself, before GPU init;
* ``config.workload`` names the per-rank kernel shape.
"""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
BENCH = os.path.join(ROOT, "bench.py")


def _json_lines(out: str):
    return [json.loads(line) for line in out.splitlines() if line.startswith("{")]


def _env():
    env = dict(os.environ)
    env.pop("WORLD_SIZE", None)
    env.pop("RANK", None)
    env.pop("LOCAL_RANK", None)
    return env


@pytest.mark.parametrize("n", [2, 4])
def test_self_launch_spawns_n_ranks_and_prints_one_line(n):
    r = subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--dry-run", "--cpu-baseline-seconds", "0.2"],
                       capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1, r.stdout
    line = lines[0]
    assert line["dry_run"] and line["n_gpus"] == n
    ranks = line["ranks"]
    assert sorted(x["rank"] for x in ranks) == list(range(n))
    assert len({x["pid"] for x in ranks}) == n  # N distinct processes
    assert all(x["pid"] != os.getpid() for x in ranks)
    cpu = line["cpu_baseline"]
    assert cpu["kind"] == "port" and cpu["cores"] == 1 and cpu["value"] > 0 and cpu["cpu_model"]
    per = 8 // n
    assert f"k_clients<float,float,{per},{8 - per}>" in line["config"]["workload"]


def test_outer_torchrun_rank0_measures_cpu_baseline():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
                        "--master-addr", "127.0.0.1", "--master-port", str(port), BENCH, "--gpus", "2",
                        "--dry-run", "--cpu-baseline-seconds", "0.2"],
                       capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = _json_lines(r.stdout)
    assert len(lines) == 1
    assert lines[0]["n_gpus"] == 2 and lines[0]["cpu_baseline"]["value"] > 0


def test_world_one_runs_in_process():
    r = subprocess.run([sys.executable, BENCH, "--dry-run", "--cpu-baseline-seconds", "0"],
                       capture_output=True, text=True, timeout=120, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = _json_lines(r.stdout)
    assert line["n_gpus"] == 1 and line["ranks"][0]["pid"] != os.getpid()
    assert line["cpu_baseline"] is None
    assert "k_clients<float,float,8,0>" in line["config"]["workload"]


@pytest.mark.parametrize("opts,expect", [
    (["--exchange", "sharded", "--gather"], "ncclReduceScatter(uint64) of the partial sum"),
    (["--shard", "elements"], "element-sharded: every rank masks its 1/2 of every client's elements"),
])
def test_exchange_options_reach_every_rank(opts, expect):
    """The N>1 exchange options (sharded server, element sharding) pass
    through the self-launcher to the ranks and name themselves in
    config.workload."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--cpu-baseline-seconds", "0", *opts],
                       capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = _json_lines(r.stdout)
    assert line["n_gpus"] == 2 and expect in line["config"]["workload"]


def test_many_client_workload_names_the_pair_shared_schedule():
    r = subprocess.run([sys.executable, BENCH, "--dry-run", "--cpu-baseline-seconds", "0", "--clients", "32",
                        "--elems", "1000"], capture_output=True, text=True, timeout=120, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = _json_lines(r.stdout)
    assert "pair-shared schedule" in line["config"]["workload"] and "24 k_clients<float,float,8,0,1>" in \
        line["config"]["workload"]


def test_bench_kernel_variant_table_matches_the_registry():
    """bench.py names the k_clients instantiation a fused launch dispatches
    (roofline.kernel); its table of sum-only shapes must be the registry's
    (sfl_amd/csrc/sa_clients_f32.hip)."""
    import re

    sys.path.insert(0, ROOT)
    import bench

    src = open(os.path.join(ROOT, "sfl_amd", "csrc", "sa_clients_f32.hip")).read()
    shapes = {(int(a), int(b)) for a, b in re.findall(r"\bSO\((\d+), (\d+)\)", src)}
    shapes |= {(int(a), int(b)) for a, b in
               re.findall(r"SA_ENTRY_K\(float, float, SA_F32, SA_F32, (\d+), (\d+), kLean1 \| kSumOnly\)", src)}
    assert shapes == bench.SUM_ONLY_SHAPES
    assert bench.kernel_variant(8, 0, False) == 4 and bench.kernel_variant(8, 0, True) == 0
    assert bench.kernel_variant(1, 7, False) == 6 and bench.kernel_variant(1, 5, False) == 2
