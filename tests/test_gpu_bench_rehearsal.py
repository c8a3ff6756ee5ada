"""The driver's N > 1 bench, rehearsed with real rank processes on the one
GPU of the test box (`bench.py --gpus W --rehearse-one-gpu`): the
self-launcher, W torchrun ranks, every design's code path in run_design
(client sharding with the pipelined sharded server, its gather, the reduce
to rank 0, element sharding with and without the gather) and the max-over-
ranks timing, with the collectives through a host stand-in (bench.HostStandinComm:
a mapping shared by the ranks, barriers included) because
RCCL refuses two ranks on one GPU ("Duplicate GPU detected",
tools/rccl_two_ranks_one_gpu.py).  RCCL itself runs at world 1 in
tests/test_gpu_rccl.py; the data path of every rank is checked against the
oracle in tests/test_gpu_dist_pipeline.py and test_gpu_world_emulation.py."""
import json
import os
import subprocess
import sys
import time

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def rehearsal_env(env: dict) -> dict:
    """Environment for W rank processes on this box's one GPU: the phase
    timeline on stderr (SFL_BENCH_TRACE), and 2 hardware queues per process
    instead of HIP's 4 (8 processes x 4-5 streams would ask the GPU's
    scheduler for 32+ queues at once, which the driver's one-process-per-GPU
    run never does)."""
    for k in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT"):
        env.pop(k, None)
    env["SFL_BENCH_TRACE"] = "1"
    env["GPU_MAX_HW_QUEUES"] = "2"
    return env


def oracle_check(C: int, n: int, fxp_bits: int = 18) -> str:
    """bench.py's round-0 result check from the oracle: the bench's synthetic
    inputs regenerated the same way (torch.Generator on the GPU), the masked
    sum = sum of the quantized vectors (the pair masks cancel), decoded, and
    the float64 bits digested by position (bench.position_digest)."""
    import numpy as np

    from oracle import secagg as o

    dev = torch.device("cuda", 0)
    s = np.zeros(n, dtype=np.uint64)
    for c in range(C):  # accumulated client by client (no C x n stack at 100M)
        g = torch.Generator(device=dev).manual_seed(20260116 + c)
        x = (torch.randn(n, generator=g, device=dev, dtype=torch.float32) * 1e-2).cpu().numpy()
        s += o.quantize(x, None, fxp_bits)
        del x
    dec = o.decode(s, fxp_bits)
    return f"{digest_np(dec):016x}"


def mix64_np(z):
    """splitmix64's finalizer in numpy uint64 (bench.mix64's definition)."""
    z = np.asarray(z, dtype=np.uint64).copy()
    z ^= z >> np.uint64(30)
    z *= np.uint64(0xBF58476D1CE4E5B9)
    z ^= z >> np.uint64(27)
    z *= np.uint64(0x94D049BB133111EB)
    z ^= z >> np.uint64(31)
    return z


def digest_np(dec, base: int = 0) -> int:
    """bench.position_digest restated in numpy: sum_i mix64(bits(dec[i])) *
    (2 (base + i) + 1) * 0x9E3779B97F4A7C15 mod 2^64."""
    idx = np.arange(base, base + dec.size, dtype=np.uint64)
    h = (idx * np.uint64(2) + np.uint64(1)) * np.uint64(0x9E3779B97F4A7C15)  # bench.CHECK_MULT
    return int(np.sum(mix64_np(np.ascontiguousarray(dec, dtype=np.float64).view(np.uint64)) * h, dtype=np.uint64))


def has_gpu() -> bool:
    """A GPU is visible -- asked without initialising HIP in this process
    (device_count does not; is_available does, on this image)."""
    return torch.cuda.device_count() > 0


def oracle_check_in_child(C: int, n: int) -> str:
    """oracle_check computed in a child process, so that THIS process (the
    test runner, which starts the rank processes) holds no GPU context while
    the W rank processes run: W + 1 > 8 processes on the one GPU run slower
    (profiles/r06/rehearsal_context_probe.txt); conftest.py runs this module
    first for the same reason -- a speed-up, the tests pass in any order."""
    code = ("import sys; sys.path[:0] = [%r, %r]; from test_gpu_bench_rehearsal import oracle_check; "
            "print(oracle_check(%d, %d))" % (os.path.join(ROOT, "tests"), ROOT, C, n))
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=170, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    return r.stdout.split()[-1]


@pytest.fixture(scope="module")
def check_1m():
    if not has_gpu():
        pytest.skip("no GPU")
    return oracle_check_in_child(8, 1000003)


@pytest.mark.parametrize("comm", ["rccl", "standin"])
@pytest.mark.parametrize("world", [2, 4, 8])
def test_bench_n_ranks_every_design(world, comm, check_1m):
    """bench.py --gpus W with every design, W rank processes on this GPU:
    comm "rccl" runs the product's RcclComm -- real RCCL collectives between
    the ranks, each its own RCCL node (NCCL_HOSTID) over the socket
    transport; "standin" the host stand-in."""
    if not has_gpu():
        pytest.skip("no GPU")
    env = rehearsal_env(dict(os.environ))
    t0, before = time.time(), host_counters()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--rehearse-one-gpu",
                        "--rehearse-comm", comm,
                        "--elems", "1000003", "--steps", "3", "--warmup", "1", "--variant-steps", "2",
                        "--host-resident-steps", "3", "--cpu-baseline-seconds", "0", "--watchdog-seconds", "150"],
                       capture_output=True, text=True, timeout=170, env=env, cwd=ROOT)
    _keep_stderr(f"every_design_w{world}_{comm}", r, t0, before=before)
    if r.returncode != 0:  # the lines that say why (ranks interleave their output), then the tail
        why = [ln for ln in r.stderr.splitlines()
               if any(k in ln for k in ("Error", "error:", "Traceback", "watchdog", "still running", "exitcode",
                                        "rank 0: phase", "headline not"))]
        rep = r.stderr[r.stderr.find("---- bench.py: rank"):] if "---- bench.py: rank" in r.stderr else ""
        pytest.fail(f"bench.py --gpus {world} --rehearse-one-gpu: rc {r.returncode} after {time.time() - t0:.0f} s\n"
                    + "\n".join(why[:60]) + "\n--- failing ranks ---\n" + rep[:8000]
                    + "\n--- stderr tail ---\n" + r.stderr[-1500:]
                    + "\n--- stdout tail ---\n" + r.stdout[-1000:])
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    line = lines[0]
    # a complete run (no design declared hung by the watchdog), with rank 0's
    # phase timeline in the message if not
    assert not line.get("variants_incomplete") and "host_resident" in line, (
        f"after {time.time() - t0:.0f} s: {line.get('exchange_variants')}\n" + _explain(r))
    # the headline is the reduce-scatter sharded server, measured first
    assert line["n_gpus"] == world and "rehearsal" in line and line["config"]["design"] == "sharded"
    assert ("RcclComm" in line["rehearsal"]) == (comm == "rccl")
    assert line["roofline"]["exchange"]["mode"] == "rehearsal" and line["roofline"]["exchange"]["bound"]
    assert "exchange_probe" not in line and line["exchange_variants"][0]["name"] == "sharded"
    # RCCL's own account (benchkit/rccl_log.py): W ranks, and the socket
    # transport the NCCL_HOSTID rehearsal forces -- so the node's first
    # record will show P2P/IPC (xGMI) by itself
    if comm == "rccl":
        rc = line["rccl"]
        assert rc["world"] == world and rc["nranks"] == world and rc["nranks_logged"] == [world], rc
        assert rc["transports"].get("NET/Socket", 0) > 0 and rc["xgmi"] is False, rc
        assert not any(k.startswith("P2P") for k in rc["transports"]), rc
        assert sorted(rc["rehearsal_env"]) == ["NCCL_HOSTID", "NCCL_IB_DISABLE", "NCCL_SOCKET_IFNAME"], rc
    else:
        assert "rccl" not in line
    # the headline with inputs and results in pinned host memory (H2D / D2H inclusive)
    hr = line["host_resident"]
    assert "error" not in hr, hr
    assert hr["grad_elems_per_s"] > 0 and hr["pcie_bytes_per_rank_per_step"]["h2d"] == 4 * (8 // world) * 1000003, hr
    # every design's round-0 result equals the oracle's (and so N = 1's)
    assert line["check"]["decoded_digest"] == check_1m and line["designs_agree"] is True
    assert all(v["check_digest"] == check_1m for v in line["exchange_variants"]), line["exchange_variants"]
    per = 8 // world
    assert line["config"]["clients_per_gpu"] == per
    assert line["roofline"]["kernel"].startswith(f"k_clients<float, float, {per}, {8 - per}, ")
    assert line["exchange"]["chunks"] == 8
    names = [v["name"] for v in line["exchange_variants"]]
    assert sorted(names) == sorted(["sharded", "sharded+gather", "direct", "reduce", "elements", "elements+gather"])
    for v in line["exchange_variants"]:
        assert v["value"] > 0 and v["kernel_ms_per_step"] > 0, v
        if v["name"].startswith("elements"):
            assert v["kernel"].startswith("k_clients<float, float, 8, 0, ")
        else:
            assert v["xchg_ms"] > 0 and v["bytes_per_rank_per_step"] > 0


def test_bench_n1_line(check_1m):
    """The driver's N = 1 bench path at a small size: one JSON line with the
    contract's fields; one launch per step timed by one event pair around
    the timed region (kernel time <= wall time per step)."""
    if not has_gpu():
        pytest.skip("no GPU")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--elems", "1000003", "--steps", "5",
                        "--warmup", "2", "--cpu-baseline-seconds", "0"],
                       capture_output=True, text=True, timeout=110, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1, r.stdout
    d = lines[0]
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "roofline", "config"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 5 and d["warmup"] == 2
    rf = d["roofline"]
    assert rf["launches_per_step"] == 1 and rf["kernel_timing"].startswith("one HIP event pair")
    assert 0 < rf["kernel_ms_per_step"] <= d["ms_per_step"] * 1.01
    assert abs(d["value"] - 8 * 1000003 / (d["ms_per_step"] / 1e3)) < 1e-6 * d["value"]
    assert d["check"]["decoded_digest"] == check_1m


def host_counters() -> dict:
    """Host-side counters that tell a stalled multi-rank run's story: the
    cgroup's CPU throttling (cgroup v2 cpu.stat) and TCP retransmissions
    (/proc/net/snmp) -- what a rank stuck in a socket wait points at."""
    out = {}
    try:
        with open("/sys/fs/cgroup/cpu.stat") as f:
            for ln in f:
                k, v = ln.split()
                if k in ("usage_usec", "nr_periods", "nr_throttled", "throttled_usec"):
                    out[k] = int(v)
    except (OSError, ValueError):
        pass
    try:
        with open("/proc/net/snmp") as f:
            rows = [ln.split() for ln in f if ln.startswith("Tcp:")]
        if len(rows) == 2:
            tcp = dict(zip(rows[0][1:], rows[1][1:]))
            out["tcp_retrans_segs"] = int(tcp.get("RetransSegs", 0))
    except (OSError, ValueError):
        pass
    return out


def _keep_stderr(name: str, r, t0: float, slow: float = 60.0, before: dict = None) -> None:
    """A failed or slow (> `slow` s) multi-rank run's whole stderr (every
    rank's phase timeline and, when the watchdog cut it, every rank's stack
    dump) to gpurun_out/rehearsal_stderr/ for reading afterwards, headed by
    the host counters' change over the run."""
    if r.returncode == 0 and time.time() - t0 < slow:
        return
    after = host_counters()
    delta = {k: after[k] - before[k] for k in after if before and k in before}
    d = os.path.join(ROOT, "gpurun_out", "rehearsal_stderr")
    os.makedirs(d, exist_ok=True)
    with open(os.path.join(d, f"{name}_{int(time.time())}.err"), "w") as f:
        f.write(f"rc {r.returncode} after {time.time() - t0:.1f} s; host counters over the run: {json.dumps(delta)}\n"
                + r.stderr)


def _explain(r) -> str:
    """A failed bench run's story: rank 0's phase timeline (SFL_BENCH_TRACE),
    the launcher's per-rank tracebacks / watchdog dumps, the stderr tail."""
    phases = [ln for ln in r.stderr.splitlines() if "rank 0: phase" in ln or "headline not" in ln]
    rep = r.stderr[r.stderr.find("---- bench.py: rank"):] if "---- bench.py: rank" in r.stderr else ""
    return "\n".join(phases) + "\n--- failing ranks ---\n" + rep[:8000] + "\n--- stderr tail ---\n" + r.stderr[-1500:]


def _rehearse(world, inject, *extra, timeout=170):
    env = rehearsal_env(dict(os.environ))
    env["SFL_BENCH_INJECT"] = inject
    t0, before = time.time(), host_counters()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(world), "--rehearse-one-gpu",
                           "--elems", "1000003", "--steps", "3", "--warmup", "1", "--variant-steps", "2",
                           "--host-resident-steps", "0", "--cpu-baseline-seconds", "0", "--watchdog-seconds", "150",
                           *extra],
                          capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    _keep_stderr(f"rehearse_{inject.replace(':', '-').replace(',', '_')}", r, t0, slow=45.0, before=before)
    return r


def test_bench_8_ranks_keeps_headline_when_designs_fail_or_hang():
    """The driver's N = 8 run cannot lose its headline to a design after it:
    `direct` raising on every rank is recorded with its error and the run
    goes on; `elements` hanging makes rank 0 print the line so far once the
    variant timeout passes, `elements+gather` marked skipped, exit 0."""
    if not has_gpu():
        pytest.skip("no GPU")
    r = _rehearse(8, "fail:direct,hang:elements", "--variant-timeout", "15")
    assert r.returncode == 0, _explain(r)
    (line,) = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert line["value"] > 0 and line["config"]["design"] == "sharded" and line["variants_incomplete"]
    got = {v["name"]: v for v in line["exchange_variants"]}
    assert got["sharded"]["value"] > 0 and got["reduce"]["value"] > 0 and got["sharded+gather"]["value"] > 0
    assert got["direct"]["error"] == "failed" and "injected failure" in got["direct"]["detail"]
    assert got["elements"]["error"] == "hung" and got["elements+gather"]["error"] == "skipped"


def test_bench_8_ranks_failing_rank_names_itself():
    """A rank that fails puts its own traceback at the end of the launcher's
    stderr (per-rank logs + torchrun's error file), not 8 ranks' banners."""
    if not has_gpu():
        pytest.skip("no GPU")
    r = _rehearse(8, "raise:rank3")
    assert r.returncode != 0
    tail = r.stderr[-3000:]
    assert "rank 3 failed" in tail and "SFL_BENCH_INJECT: rank 3 fails at start-up" in tail, tail


@pytest.fixture(scope="module")
def check_100m():
    if not has_gpu():
        pytest.skip("no GPU")
    return oracle_check_in_child(8, 100_000_000)


def _full_size_line(*extra, timeout=150):
    env = rehearsal_env(dict(os.environ))
    t0 = time.time()
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--steps", "1", "--warmup", "0",
                        "--cpu-baseline-seconds", "0", "--variants", "none", "--host-resident-steps", "0", *extra],
                       capture_output=True, text=True, timeout=timeout, env=env, cwd=ROOT)
    _keep_stderr("full_size" + ("_w8" if "--gpus" in extra else "_n1"), r, t0, slow=40.0)
    assert r.returncode == 0, _explain(r)
    (line,) = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    return line


def test_full_size_check_n1_vs_oracle(check_100m):
    """The driver's N = 1 configuration at the headline size (8 x 100M): the
    line's round-0 digest equals the oracle's (the bench's synthetic inputs,
    quantized and summed by numpy: the masks cancel)."""
    assert _full_size_line()["check"]["decoded_digest"] == check_100m


def test_full_size_check_n8_rehearsal_vs_oracle(check_100m):
    """The N = 8 configuration at the headline size, rehearsed on this GPU (8
    rank processes, <1,7> lean launches, the 8-chunk pipelined sharded server
    over real RCCL reduce-scatters between the ranks): the same digest as the
    oracle's and N = 1's -- the value the driver's SCALE lines must print."""
    line = _full_size_line("--gpus", "8", "--rehearse-one-gpu", "--watchdog-seconds", "140")
    assert line["check"]["decoded_digest"] == check_100m and line["config"]["clients_per_gpu"] == 1
