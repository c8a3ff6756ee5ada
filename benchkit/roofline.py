"""bench.py's roofline fields: the HBM and VALU peaks, the committed
rocprofv3 PMC passes (HBM bytes and VALU instructions per launch of the
exact kernel instantiation, scaled to the run's launch size), and the
same-box draw-loop ceilings of tools/microbench/draw_issue."""

from __future__ import annotations

import json
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


HBM_PEAK_GBPS = 8000.0          # MI355X HBM3E spec (MI355X_MICROARCH.md)
# PCG64 draw-loop ceilings (tools/microbench/draw_issue.hip,
# profiles/r01/draw_issue_microbench.txt), the draw loop alone with the
# product kernel's operand layout and schedule; the first is measured live on
# the bench's own box when the tool is built (draw_loop_ceilings), this
# constant is the fallback:
PCG_PAIR_DRAWS_2WAVE = 1.34e12  # pair draws (both ends accumulated), 2 waves/SIMD = the L=8 kernel's
                                # occupancy ("dual pair28 E2", best of 1.29-1.34e12 run to run)
PCG_ONE_DRAWS_8WAVE = 1.57e12   # one-sided draws at 8 waves/SIMD ("dual one7 E2")


PMC_DIRS = [os.path.join(ROOT, "profiles", r) for r in ("r06", "r05", "r04", "r03", "r02", "r01")]  # newest first
PMC_ELEMS = 100_000_000  # element positions per launch of the committed PMC passes


def kernel_key(name: str):
    """The instantiation a PMC row belongs to: (L, X, K) of a k_clients kernel
    (K, the variant flags of sa_internal.h, is 0 in round-1 names that carry
    none), otherwise the bare kernel name.  The variant decides the bytes:
    k_clients<8, 0, 1> (kBipartite, masks only) moves 16 B per element
    position, k_clients<8, 0, 4> (kSumOnly) 40 B."""
    import re

    m = re.search(r"k_clients<float, float, (\d+), (\d+)(?:, (\d+))?>", name)
    if m:
        return ("k_clients", int(m.group(1)), int(m.group(2)), int(m.group(3) or 0))
    name = name.strip()
    if name.startswith("void "):
        name = name[5:]
    return name.split("(")[0].strip()


def pmc_traffic(kernel: str, elems_per_launch: int, pmc_elems: int = PMC_ELEMS) -> dict | None:
    """HBM bytes per launch of `kernel` from the committed rocprofv3 PMC passes
    (tools/gpu_profile.sh: separate FETCH_SIZE / WRITE_SIZE runs of
    tools/kernel_bench.py, every per-rank shape at 100M element positions per
    launch), scaled to this run's launch size (the kernel streams: its bytes
    are linear in the element count).  Rows are matched on the kernel's full
    instantiation (kernel_key).  Units are KiB; gfx950 reports FETCH_SIZE at
    half the bytes of 16-B/lane streaming reads, so it is doubled
    (MI355X_MICROARCH.md, HBM); both corrections were checked on the
    k_sum_u64 calibration launch in the same runs (known bytes)."""
    import csv

    want = kernel_key(kernel)
    for d in PMC_DIRS:
        vals = {}
        for counter, fname, scale in (("FETCH_SIZE", "pmc_fetch_size.csv", 2.0),
                                      ("WRITE_SIZE", "pmc_write_size.csv", 1.0)):
            path = os.path.join(d, fname)
            if not os.path.exists(path):
                break
            with open(path) as f:
                v = [float(r["Counter_Value"]) for r in csv.DictReader(f)
                     if r["Counter_Name"] == counter and kernel_key(r["Kernel_Name"]) == want]
            if not v:
                break
            vals[counter] = scale * 1024.0 * sum(v) / len(v) * elems_per_launch / pmc_elems
        if len(vals) == 2:
            return {"bytes": vals["FETCH_SIZE"] + vals["WRITE_SIZE"], "read": vals["FETCH_SIZE"],
                    "write": vals["WRITE_SIZE"], "rows_matched": kernel_key(kernel),
                    "source": os.path.relpath(d, ROOT) + "/pmc_{fetch,write}_size.csv",
                    "scaled_from_elems": pmc_elems}
    return None


VALU_PEAK_WAVE_INSTR_PER_S = 1024 * 2.4e9 / 4  # 256 CUs x 4 SIMDs, one wave64 VALU instruction per 4 cycles
                                               # at the 2.4 GHz peak engine clock (MI355X_MICROARCH.md)


def pmc_valu(kernel: str, elems_per_launch: int, pmc_elems: int = PMC_ELEMS) -> dict | None:
    """VALU wave instructions per launch of `kernel` from the committed SQ
    census (tools/pmc_sq.sh: SQ_INSTS_VALU on tools/kernel_bench.py launches
    of 100M element positions), matched on the full instantiation and scaled
    to this run's launch size -- SURVEY.md 8(d)'s "achieved int-op rate"."""
    import csv

    want = kernel_key(kernel)
    for d in PMC_DIRS:
        path = os.path.join(d, "pmc_sq_census.csv")
        if not os.path.exists(path):
            continue
        with open(path) as f:
            v = [float(r["Counter_Value"]) for r in csv.DictReader(f)
                 if r["Counter_Name"] == "SQ_INSTS_VALU" and kernel_key(r["Kernel_Name"]) == want]
        if v:
            return {"valu_wave_instr": sum(v) / len(v) * elems_per_launch / pmc_elems,
                    "source": os.path.relpath(path, ROOT) + " (SQ_INSTS_VALU)", "scaled_from_elems": pmc_elems}
    return None


def traffic_field(pmc: dict | None, alg_bytes_per_launch: float):
    """roofline.traffic from the PMC bytes: never a figure below the
    algorithmic bytes without saying so (HBM traffic under the bytes the
    launch must move means the rows belong to another kernel, or the
    kernel skipped work) -- such a figure is withheld (None) with a note."""
    if pmc is None:
        return None, None
    if pmc["bytes"] < 0.98 * alg_bytes_per_launch:
        return None, dict(pmc, note=f"PMC bytes {pmc['bytes']:.4g} below the algorithmic "
                                    f"{alg_bytes_per_launch:.4g} B per launch: withheld")
    return pmc["bytes"], pmc


def _draw_issue(case: str, waves: int, local_rank: int | None) -> dict | None:
    import subprocess

    exe = os.path.join(ROOT, "tools", "microbench", "draw_issue")
    if not os.path.exists(exe):
        return None
    env = dict(os.environ)
    if local_rank is not None:  # this rank's GPU only (an index into the visible list)
        vis = [v for v in env.get("HIP_VISIBLE_DEVICES", "").split(",") if v]
        env["HIP_VISIBLE_DEVICES"] = vis[local_rank] if local_rank < len(vis) else str(local_rank)
    try:
        r = subprocess.run([exe, case, str(waves)], capture_output=True, text=True, timeout=120, env=env)
        line = [ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1]
        return json.loads(line)
    except (subprocess.SubprocessError, IndexError, ValueError, OSError):
        return None


def draw_loop_ceilings(local_rank: int | None = None) -> dict:
    """The PCG64 draw loop alone with the masking kernel's operand layout and
    schedule (tools/microbench/draw_issue: median of 15 launches after 40
    warm-up ones), measured on THIS rank's GPU in a child process before this
    process touches the GPU, so roofline.valu compares the kernel with a
    same-box ceiling (boards differ by a few % in clock under the power
    limit): pair draws ("dual pair28 E2" at the 8-client kernel's 2
    waves/SIMD) and one-sided draws ("dual one7 E2" at 8 waves/SIMD, the
    cross streams' kind).  Missing entries if the tool is absent or fails."""
    out = {}
    for kind, case, w in (("pair", "dual pair28 E2", 2), ("one", "dual one7 E2", 8)):
        r = _draw_issue(case, w, local_rank)
        if r:
            out[kind] = r
    return out


# ---------------------------------------------------------------------------
# N > 1: the exchange step against the xGMI links
# ---------------------------------------------------------------------------
XGMI_LINK_GBPS_PER_DIRECTION = 76.5
XGMI_SOURCE = ("the task brief's MI355X node figure, 7 xGMI links x ~153 GB/s per GPU, read as both directions "
               "of a link together (76.5 GB/s each way; if 153 is per direction every link_frac halves); "
               "MI355X_MICROARCH.md states no xGMI figure")


def exchange_model(design: str, world: int, n_elems: int, kernel_ms: float, xchg_ms: float, chunks: int,
                   mode: str = "measured") -> dict | None:
    """The N > 1 step as DESIGN.md §5 models it: per rank, the masking
    kernel of its shape, and the exchange's bytes on its busiest directed
    xGMI link, with chunk j's exchange overlapping chunk j+1's masking:

        predicted_ms_per_step = max(kernel, link) + min(kernel, link) / chunks

    ``link`` = bytes on the busiest directed link / the per-link peak.  The
    replaced transfer is the reference's masked-vector ``.to(server)``
    (sfl/distributed/op_strategy.py:131-141, sparse_plain_aggregator.py:86).
    ``mode``: "measured" (the driver's node), "rehearsal" (one GPU, host
    stand-ins: the fields are the model's, the timings not xGMI's) or
    "dry-run" (no GPU).  None at world 1 or without an exchange."""
    if world <= 1 or design == "elements":
        return None
    n = int(n_elems)
    if design in ("sharded", "direct"):
        per_link = 8 * n / world
        what = ("every rank's uint64 partial-sum shard for each peer crosses one link (all W-1 links of a GPU "
                "busy, both directions): 8N/W bytes per directed link")
    elif design == "sharded+gather":
        per_link = 16 * n / world
        what = ("8N/W bytes of uint64 shard per directed link, then the float64 shards gathered into rank 0 "
                "(another 8N/W on each of its in-links)")
    elif design == "elements+gather":
        per_link = 8 * n / world
        what = "no exchange for the sum; the float64 slices gathered into rank 0: 8N/W bytes per in-link"
    elif design == "reduce":
        per_link = 8 * n
        what = "ncclReduce to rank 0: the full 8N-byte partial sum passes each link of the reduction ring"
    else:
        return None
    peak = XGMI_LINK_GBPS_PER_DIRECTION
    link_ms = per_link / (peak * 1e9) * 1e3
    chunks = max(1, int(chunks))
    if kernel_ms is None:
        predicted = None
    else:
        predicted = max(kernel_ms, link_ms) + min(kernel_ms, link_ms) / chunks
    achieved = per_link / (xchg_ms / 1e3) / 1e9 if xchg_ms and xchg_ms > 0 else None
    return {"mode": mode, "bytes_per_link_per_step": per_link, "schedule": what,
            "peak_GBps_per_link_direction": peak, "peak_source": XGMI_SOURCE,
            "link_ms_at_peak": link_ms, "kernel_ms_per_step": kernel_ms, "exchange_ms_per_step": xchg_ms,
            "achieved_GBps_per_link": achieved, "link_frac": achieved / peak if achieved else None,
            "predicted_ms_per_step": predicted,
            "bound": None if kernel_ms is None else ("link" if link_ms > kernel_ms else "kernel"),
            "note": ("exchange_ms_per_step is the comm stream's time per step (HIP events, max over ranks); "
                     "achieved_GBps_per_link = bytes_per_link_per_step / that time")}


def committed_kernel_ms(clients: int, world: int, n_elems: int) -> tuple[float | None, str | None]:
    """Rank 0's masking-kernel time per step for C clients over W GPUs from
    the newest committed tools/kernel_bench.py run (scaled linearly from its
    element count), for --dry-run's exchange model; (None, None) if absent."""
    for d in PMC_DIRS:
        path = os.path.join(d, "kernel_bench_shapes.json")
        if not os.path.exists(path):
            continue
        with open(path) as f:
            kb = json.load(f)
        for c in kb.get("cases", []):
            if c.get("C") == clients and c.get("W") == world and c.get("path") == "fused":
                return c["ms_median"] * n_elems / kb["elems"], os.path.relpath(path, ROOT)
    return None, None
