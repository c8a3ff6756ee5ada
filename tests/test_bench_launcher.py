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
    r = subprocess.run([sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", "2",
                        "--rdzv-backend", "c10d", "--rdzv-endpoint", "127.0.0.1:0", "--rdzv-id", "outer-test",
                        "--local-addr", "127.0.0.1", BENCH, "--gpus", "2",
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
    (["--exchange", "reduce"], "ncclReduce(uint64) of the partial sum to rank 0"),
    (["--exchange", "direct"], "direct shard transfers (ncclSend/Recv, uint64) of the partial sum"),
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


def test_n_gt_1_line_names_every_exchange_design_and_a_safe_launch():
    """One `bench.py --gpus N` run times every N>1 design in the same process
    group (exchange_variants, the headline first); the ranks rendezvous on a
    port the store bound itself (no port probe); the watchdog fires before the
    driver's 600 s lease."""
    import bench

    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--cpu-baseline-seconds", "0"],
                       capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = _json_lines(r.stdout)
    names = [v["name"] for v in line["exchange_variants"]]
    assert names[0] == "sharded" and sorted(names) == sorted(bench.VARIANTS) and len(names) >= 3
    assert "ncclReduceScatter(uint64) of the partial sum" in line["config"]["workload"]
    ports = {x["master_port"] for x in line["ranks"]}
    assert len(ports) == 1 and None not in ports
    assert 0 < line["watchdog_seconds"] < 600
    src = open(os.path.join(ROOT, "benchkit", "launcher.py")).read()
    assert ".bind(" not in src and "--master-port" not in src.split("def launch_ranks")[1].split("def ")[0]
    # a subset, and the headline taken from the flags
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--cpu-baseline-seconds", "0",
                        "--exchange", "reduce", "--variants", "elements"],
                       capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = _json_lines(r.stdout)
    assert [v["name"] for v in line["exchange_variants"]] == ["reduce", "elements"]


def test_pmc_traffic_keys_on_the_full_instantiation():
    """roofline.traffic comes from the committed PMC rows of exactly the
    kernel the bench times: every k_clients instantiation the bench can name
    resolves to rows of its own (L, X, K), whose bytes are the launch's
    algorithmic bytes (4 L N read + 8 N written), never the average with
    another variant's rows (the bipartite <8,0,1> masks-only launch moves
    16 B per element position, the sum-only <8,0,4> 40 B)."""
    import csv

    import bench

    n = 10 ** 8
    for L in (8, 4, 2, 1):  # the per-rank shapes of N = 1, 2, 4, 8
        X = 8 - L
        k = bench.kernel_variant(L, X, False)
        name = f"void sa::k_clients<float, float, {L}, {X}, {k}>"
        p = bench.pmc_traffic(name, n)
        assert p is not None, name
        assert p["rows_matched"] == ("k_clients", L, X, k)
        alg = 4 * L * n + 8 * n
        assert abs(p["bytes"] - alg) / alg < 0.01, (name, p["bytes"], alg)
        assert bench.traffic_field(p, alg)[0] == p["bytes"]
    p = bench.pmc_traffic("void sa::k_clients<float, float, 8, 0, 4>", n)
    assert abs(p["bytes"] - 4.0e9) / 4.0e9 < 1e-3
    b = bench.pmc_traffic("void sa::k_clients<float, float, 8, 0, 1>", n)
    assert abs(b["bytes"] - 1.6e9) / 1.6e9 < 0.01
    # every kernel row in the committed files resolves to rows of its own key only
    for d in bench.PMC_DIRS:
        path = os.path.join(d, "pmc_fetch_size.csv")
        if not os.path.exists(path):
            continue
        with open(path) as f:
            keys = {bench.kernel_key(r["Kernel_Name"]) for r in csv.DictReader(f) if "sa::" in r["Kernel_Name"]}
        assert len(keys) >= 2
    # a figure below the algorithmic bytes is withheld, with a note
    t, detail = bench.traffic_field({"bytes": 2.8e9, "read": 2.0e9, "write": 0.8e9}, 4.0e9)
    assert t is None and "withheld" in detail["note"]


def test_pmc_valu_reads_the_census_of_the_timed_kernel():
    """roofline.valu.issue: VALU wave instructions per launch from the
    committed SQ census of exactly the timed instantiation, scaled to the
    launch size; ~27 per pair draw for the 8-client launch."""
    import bench

    n = 10 ** 8
    v = bench.pmc_valu("void sa::k_clients<float, float, 8, 0, 4>", n)
    assert v is not None
    per_pair_draw = v["valu_wave_instr"] / (28 * n / 64)
    assert 24 < per_pair_draw < 30, per_pair_draw
    half = bench.pmc_valu("void sa::k_clients<float, float, 8, 0, 4>", n // 2)
    assert abs(half["valu_wave_instr"] * 2 - v["valu_wave_instr"]) < 1
    assert bench.pmc_valu("void sa::k_clients<float, float, 3, 5, 4>", n) is None


def _dry(n, inject, *extra):
    env = _env()
    env["SFL_BENCH_INJECT"] = inject
    return subprocess.run([sys.executable, BENCH, "--gpus", str(n), "--dry-run", "--cpu-baseline-seconds", "0",
                           "--steps", "3", "--warmup", "1", *extra],
                          capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)


def test_failed_design_is_recorded_and_the_run_goes_on():
    """A design after the headline that raises on every rank is recorded in
    its exchange_variants entry (with the error) and the next design runs;
    the headline value stands, exactly one line, exit 0."""
    r = _dry(2, "fail:direct")
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = _json_lines(r.stdout)
    assert line["value"] > 0 and line["config"]["design"] == "sharded" and not line.get("variants_incomplete")
    got = {v["name"]: v for v in line["exchange_variants"]}
    assert got["direct"]["error"] == "failed" and "injected failure in design 'direct'" in got["direct"]["detail"]
    assert got["reduce"]["value"] > 0 and got["elements+gather"]["value"] > 0


def test_hung_design_prints_the_line_so_far():
    """A design that hangs past --variant-timeout: rank 0's watchdog prints
    the line built so far (the headline and the designs before the hang),
    the hung design marked, the rest skipped; every rank exits 0."""
    r = _dry(2, "hang:elements", "--variant-timeout", "4")
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = _json_lines(r.stdout)
    assert line["value"] > 0 and line["variants_incomplete"]
    got = {v["name"]: v for v in line["exchange_variants"]}
    assert got["sharded"]["value"] > 0 and got["reduce"]["value"] > 0
    assert got["elements"]["error"] == "hung" and got["elements+gather"]["error"] == "skipped"


def test_design_failing_on_one_rank_names_the_rank():
    """A design raising on ONE rank leaves its peers in the design's
    collectives: the watchdog declares it hung and the line carries the
    failing rank's error (published through the c10d store)."""
    r = _dry(2, "fail:reduce@1", "--variant-timeout", "4")
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = _json_lines(r.stdout)
    got = {v["name"]: v for v in line["exchange_variants"]}
    assert got["reduce"]["error"] == "hung" and "rank 1: RuntimeError" in got["reduce"]["detail"]
    assert got["elements"]["error"] == "skipped" and got["direct"]["value"] > 0


def test_failing_rank_prints_its_traceback_last():
    """A rank that fails at start-up: the launcher's stderr ends with that
    rank's traceback (per-rank logs / torchrun's error file), rc != 0."""
    r = _dry(4, "raise:rank3")
    assert r.returncode != 0
    tail = r.stderr[-2500:]
    assert "rank 3 failed" in tail and "SFL_BENCH_INJECT: rank 3 fails at start-up" in tail, tail
    assert not _json_lines(r.stdout)


def test_injection_parser():
    import bench

    os.environ["SFL_BENCH_INJECT"] = "fail:direct@2,hang:elements,raise:rank3"
    try:
        assert bench.injected("fail", "direct", 2) and not bench.injected("fail", "direct", 1)
        assert bench.injected("hang", "elements", 0) and bench.injected("hang", "elements", 7)
        assert not bench.injected("hang", "elements+gather", 0)
        assert bench.injected("raise", None, 3) and not bench.injected("raise", None, 0)
    finally:
        del os.environ["SFL_BENCH_INJECT"]
    assert not bench.injected("fail", "direct", 0)


def test_design_with_a_different_result_is_flagged():
    """Every design's round-0 result check must equal the headline's; one
    that differs is marked (mismatch) and the line says designs_agree false."""
    r = _dry(2, "corrupt:direct@1")
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = _json_lines(r.stdout)
    got = {v["name"]: v for v in line["exchange_variants"]}
    assert "mismatch" in got["direct"] and "mismatch" not in got["reduce"]
    assert line["designs_agree"] is False
    r = _dry(2, "")
    (line,) = _json_lines(r.stdout)
    assert line["designs_agree"] is True and all("mismatch" not in v for v in line["exchange_variants"])


def test_multi_launch_plan_names_config5_schedule():
    """Per-rank shapes beyond one launch (sum only): the first launch takes
    the internal pairs + X1 cross streams per client, masks-only launches of
    kCrossCounts the rest -- every cross stream exactly once; config 5 at 8
    GPUs is <4,4> + 3 x 32, and --clients 32 --gpus 8 names it."""
    import bench

    assert bench.multi_launch_plan(4, 28) == (4, [32, 32, 32])
    assert bench.multi_launch_plan(8, 24) == (0, [32] * 6)
    assert bench.multi_launch_plan(4, 4) is None and bench.multi_launch_plan(16, 16) is None
    for L in range(1, 9):
        for X in range(0, 60):
            p = bench.multi_launch_plan(L, X)
            if p is None:
                continue
            x1, sizes = p
            pi = L * (L - 1) // 2
            assert pi + L * x1 <= 32 and (L, x1) in bench.SUM_ONLY_SHAPES
            assert sum(sizes) == L * (X - x1) and all(c in bench.CROSS_COUNTS for c in sizes)
    r = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--dry-run", "--cpu-baseline-seconds", "0",
                        "--clients", "32", "--elems", "1000", "--steps", "1", "--warmup", "0", "--variants", "none"],
                       capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = _json_lines(r.stdout)
    assert "pair-shared multi-launch schedule: k_clients<float,float,4,4>" in line["config"]["workload"]
    assert "X = 32+32+32" in line["config"]["workload"]


def test_cross_only_counts_match_the_registry():
    """bench.CROSS_COUNTS mirrors kCrossCounts, and every count is instantiated."""
    import re

    import bench

    hdr = open(os.path.join(ROOT, "sfl_amd", "csrc", "sa_internal.h")).read()
    counts = tuple(int(v) for v in re.search(r"kCrossCounts\[\] = \{([^}]*)\}", hdr).group(1).split(","))
    assert counts == bench.CROSS_COUNTS
    src = open(os.path.join(ROOT, "sfl_amd", "csrc", "sa_clients_f32.hip")).read()
    assert {int(v) for v in re.findall(r"\bXO\((\d+)\)", src)} == set(counts)


def test_position_digest_matches_numpy_and_sees_permutations():
    """bench.position_digest (the round-0 result check): sum of
    mix64(bits(x[i])) * (2(base+i)+1) * CHECK_MULT mod 2^64, additive over
    slices at their global offsets (how the ranks' parts combine), and
    changed by swapping two shards (an XOR or a plain sum would not be)."""
    import numpy as np
    import torch

    import bench
    from test_gpu_bench_rehearsal import digest_np, mix64_np

    # mix64 is splitmix64's finalizer bit for bit (int64 tensor vs uint64 numpy)
    rng = np.random.default_rng(3)
    z = rng.integers(0, 2**64, 4096, dtype=np.uint64)
    z[:4] = [0, 1, 2**63, 2**64 - 1]
    assert np.array_equal(bench.mix64(torch.from_numpy(z.view(np.int64))).numpy().view(np.uint64), mix64_np(z))
    x = (rng.integers(-2**15, 2**15, 1_000_003) / 2.0**18).astype(np.float64)
    want = digest_np(x)
    t = torch.from_numpy(x)
    assert bench.position_digest(t, 0) == want
    k = 400_001
    assert (bench.position_digest(t[:k], 0) + bench.position_digest(t[k:], k)) % 2**64 == want
    y = np.concatenate([x[k:2 * k], x[:k], x[2 * k:]])  # two shards swapped
    assert bench.position_digest(torch.from_numpy(y), 0) != want


def test_position_digest_has_64_live_bits():
    """decoded fixed-point values k / 2^18 (|k| < 2^16)
    have >= 36 trailing zero bits in their float64 patterns, so a digest of
    the raw bits was one too and swapping two elements 2^27 apart (weights
    differing by 2^28 * CHECK_MULT) could not change it.  With mix64 neither
    holds."""
    import numpy as np
    import torch

    import bench

    rng = np.random.default_rng(7)
    for _ in range(4):
        x = (rng.integers(-2**15, 2**15, 100_003) / 2.0**18).astype(np.float64)
        assert np.all(np.bitwise_and(x.view(np.uint64), np.uint64(2**36 - 1)) == 0)  # the raw patterns
        d = bench.position_digest(torch.from_numpy(x), 0)
        assert d & (2**36 - 1) != 0
    # elements a and b swapped between positions i and i + 2^27: the parts at
    # those global positions (base) differ, as the full vectors' digests would
    a, b = torch.tensor([0.125 + 3 / 2**18], dtype=torch.float64), torch.tensor([-7 / 2**18], dtype=torch.float64)
    i, j = 12345, 12345 + 2**27
    before = (bench.position_digest(a, i) + bench.position_digest(b, j)) % 2**64
    after = (bench.position_digest(b, i) + bench.position_digest(a, j)) % 2**64
    assert before != after
    # (the old raw-bit digest could not see it: the difference was a multiple of 2^64)
    raw = lambda v, base: int(v.view(torch.int64)) * (2 * base + 1) * bench.CHECK_MULT  # noqa: E731
    assert (raw(a, i) + raw(b, j) - raw(b, i) - raw(a, j)) % 2**64 == 0


def test_importing_the_bench_loads_no_torch():
    """The self-launcher process must not touch the GPU before it starts its
    rank processes (nothing may be exec'd from a process that initialised
    HIP): importing bench.py and benchkit/ loads no torch."""
    code = ("import sys; sys.path.insert(0, %r); import bench, benchkit.launcher, benchkit.containment, "
            "benchkit.standin, benchkit.roofline, benchkit.baseline; "
            "assert 'torch' not in sys.modules, sorted(m for m in sys.modules if m.startswith('torch'))[:5]" % ROOT)
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, timeout=60, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]


def test_gpu_context_guard_reads_proc(tmp_path):
    """benchkit.launcher.gpu_context_holders (the --rehearse-one-gpu warning):
    finds a process by an open device node in /proc/<pid>/fd, here a file
    standing in for /dev/kfd, without touching the GPU."""
    from benchkit.launcher import gpu_context_holders, rehearsal_warning

    dev = tmp_path / "kfd"
    dev.write_bytes(b"")
    assert gpu_context_holders([os.getpid()], str(dev)) == []
    with open(dev) as f:
        assert gpu_context_holders([os.getpid(), os.getppid(), 2**22 + 7], str(dev)) == [os.getpid()]
        del f
    assert "9 processes on the one GPU" in rehearsal_warning([123], 8)


def test_dry_run_n8_line_carries_the_exchange_model():
    """at N > 1 the line says by itself whether the step
    is link- or kernel-bound -- roofline.exchange with the bytes per link,
    the assumed per-link peak and its source, and the predicted step from
    the rank's kernel time (--dry-run: the committed per-rank kernel time)."""
    r = subprocess.run([sys.executable, BENCH, "--gpus", "8", "--dry-run", "--cpu-baseline-seconds", "0",
                        "--steps", "1", "--warmup", "0"],
                       capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = _json_lines(r.stdout)
    m = line["roofline"]["exchange"]
    assert m["mode"] == "dry-run" and m["bytes_per_link_per_step"] == 8 * 100_000_000 / 8
    assert m["peak_GBps_per_link_direction"] > 0 and "xGMI" in m["peak_source"]
    assert m["kernel_ms_per_step"] and m["predicted_ms_per_step"] >= max(m["kernel_ms_per_step"], m["link_ms_at_peak"])
    assert m["bound"] in ("link", "kernel")
    models = {v["name"]: v["exchange_model"] for v in line["exchange_variants"]}
    assert models["elements"] is None and models["reduce"]["bytes_per_link_per_step"] == 8 * 100_000_000
    import benchkit.roofline as R

    assert R.exchange_model("sharded", 1, 10, 1.0, 1.0, 8) is None
    mm = R.exchange_model("direct", 4, 10**8, 0.9, 3.0, 8, "rehearsal")
    assert mm["link_frac"] == pytest.approx(2e8 / 3e-3 / 1e9 / R.XGMI_LINK_GBPS_PER_DIRECTION)


def _dry_ranks(extra):
    r = subprocess.run([sys.executable, BENCH, "--gpus", "2", "--dry-run", "--cpu-baseline-seconds", "0",
                        "--variants", "none", "--steps", "2", "--warmup", "1", *extra],
                       capture_output=True, text=True, timeout=240, env=_env(), cwd=ROOT)
    assert r.returncode == 0, r.stderr[-2000:]
    (line,) = _json_lines(r.stdout)
    return line["ranks"]


def test_product_ranks_never_set_the_rehearsal_rccl_env():
    """only --rehearse-one-gpu may set NCCL_HOSTID /
    NCCL_SOCKET_IFNAME / NCCL_IB_DISABLE (each rank its own RCCL node over
    sockets); the product's N > 1 ranks -- self-launched here -- set none of
    them and inherit none from the launcher, but do route RCCL's init log to
    a per-rank file (the line's rccl record)."""
    from benchkit.rccl_log import REHEARSAL_ONLY_ENV

    env = _env()
    leaked = [k for k in REHEARSAL_ONLY_ENV if k in env]
    if leaked:
        pytest.skip(f"the test environment itself sets {leaked}")
    for r in _dry_ranks([]):
        assert not set(r["comm_env"]) & set(REHEARSAL_ONLY_ENV), r
        assert r["inherited_rehearsal_env"] == [], r
        assert {"NCCL_DEBUG", "NCCL_DEBUG_SUBSYS", "NCCL_DEBUG_FILE"} <= set(r["comm_env"]), r
    for r in _dry_ranks(["--rehearse-one-gpu"]):
        assert set(REHEARSAL_ONLY_ENV) <= set(r["comm_env"]), r
    for r in _dry_ranks(["--rehearse-one-gpu", "--rehearse-comm", "standin"]):
        assert r["comm_env"] == [], r


def test_rank_comm_env_table():
    import argparse

    sys.path.insert(0, ROOT)
    import bench

    a = argparse.Namespace(rehearse_one_gpu=False, rehearse_comm="rccl")
    assert bench.rank_comm_env(a, 0, False, "/x") == {}
    env = bench.rank_comm_env(a, 3, True, "/x")
    assert env["NCCL_DEBUG_FILE"] == "/x/rank3.%p.log" and "NCCL_HOSTID" not in env
    a.rehearse_one_gpu = True
    assert bench.rank_comm_env(a, 1, True, "/x")["NCCL_HOSTID"] == "sfl-onegpu-rank1"
    a.rehearse_comm = "standin"
    assert bench.rank_comm_env(a, 1, True, "/x") == {}


# RCCL init-log lines in the formats RCCL/NCCL 2.x print (transport/p2p.cc,
# net.cc, shm.cc, init.cc); the one-GPU rehearsal's real log is checked on
# the GPU (tests/test_gpu_bench_rehearsal.py)
_LOG = """\
box:123:123 [0] NCCL INFO Channel 00/0 : 0[0] -> 1[1] via P2P/IPC/read
box:123:123 [0] NCCL INFO Channel 01/0 : 0[0] -> 1[1] via P2P/IPC/read comm 0x55d0 nRanks 02
box:123:123 [0] NCCL INFO Channel 02/0 : 0[0] -> 1[1] via P2P/direct pointer/read
box:123:123 [0] NCCL INFO Channel 00/0 : 1[1] -> 0[0] [send] via NET/Socket/0
box:123:123 [0] NCCL INFO Channel 00/0 : 1[1] -> 0[0] [receive] via NET/Socket/0
box:123:123 [0] NCCL INFO Channel 00 : 0[0] -> 1[1] via SHM/direct/direct
box:123:123 [0] NCCL INFO comm 0x55d0 rank 0 nRanks 8 nNodes 1 localRanks 8 localRank 0 MNNVL 0
box:123:123 [0] NCCL INFO ncclCommInitRank comm 0x55d0 rank 0 nranks 8 cudaDev 0 busId 5000 - Init COMPLETE
box:123:123 [0] NCCL INFO Connected all rings
unrelated line via P2P/IPC, no info tag
"""


def test_rccl_log_parse_and_combine():
    from benchkit import rccl_log as R

    s = R.summarise(_LOG)
    assert s["transports"] == {"P2P/IPC": 2, "P2P/direct pointer": 1, "NET/Socket": 2, "SHM/direct": 1}
    assert s["nranks"] == [2, 8] and s["nnodes"] == [1] and s["lines"] == 9
    xgmi_only = {"transports": {"P2P/IPC": 24}, "nranks": [8], "nnodes": [1], "lines": 40}
    per = [{"rank": r, "comm": {"nranks": 8, "rank": r, "device": r}, "log": xgmi_only} for r in range(8)]
    c = R.combine(per, 8)
    assert c["xgmi"] is True and c["nranks"] == 8 and c["transports"] == {"P2P/IPC": 192}
    assert c["devices"] == list(range(8)) and c["nnodes_logged"] == [1]
    per[3]["log"] = s
    assert R.combine(per, 8)["xgmi"] is False
    none = [{"rank": 0, "comm": None, "log": None}]
    assert R.combine(none, 1)["xgmi"] is None


def test_rccl_debug_env_respects_a_caller_log(monkeypatch):
    from benchkit import rccl_log as R

    monkeypatch.setenv("NCCL_DEBUG", "VERSION")  # what the GPU box exports: too quiet for the record
    assert R.debug_env(0, "/x")["NCCL_DEBUG"] == "INFO"
    monkeypatch.setenv("NCCL_DEBUG", "trace")
    assert R.debug_env(0, "/x")["NCCL_DEBUG"] == "TRACE"

    monkeypatch.setenv("NCCL_DEBUG_FILE", "/somewhere/else.log")
    assert R.debug_env(0, "/x") == {}
    rec = R.rank_summary(0, None, {"nranks": 2})
    assert rec["log"] is None and "NCCL_DEBUG_FILE" in rec["note"]


def test_rccl_log_parse_real_rehearsal_log():
    """A real RCCL init log (rank 0 of `bench.py --gpus 2 --rehearse-one-gpu`
    on the MI355X box, NCCL_DEBUG=INFO via benchkit/rccl_log.py): torch's
    process group and our RcclComm, two ranks, each its own RCCL node over
    sockets (NCCL_HOSTID) -- the parser sees only NET/Socket connections."""
    from benchkit import rccl_log as R

    text = open(os.path.join(ROOT, "tests", "golden", "rccl_init_rehearsal_w2_rank0.log")).read()
    s = R.summarise(text)
    assert set(s["transports"]) == {"NET/Socket"} and s["transports"]["NET/Socket"] >= 8
    assert s["nranks"] == [2] and s["nnodes"] == [2]
    c = R.combine([{"rank": 0, "comm": {"nranks": 2, "rank": 0, "device": 0}, "log": s}], 2)
    assert c["xgmi"] is False and c["nranks"] == 2
