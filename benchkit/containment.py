"""bench.py's failure containment for N > 1: fault injection, the watchdog,
errors published to the c10d store, and the contained runs of every design
after the headline."""

from __future__ import annotations

import json
import os
import sys
import time


# ------------------------------------------------ failure containment (N > 1)
#
# The driver's N > 1 run is the only place the exchange designs meet xGMI, so
# one bad design must not cost the line: the headline (the reduce-scatter
# sharded server, the design with the most evidence) runs FIRST, every other
# design runs inside `run_variants` (an exception is recorded in its
# exchange_variants entry; the ranks agree over a gloo control group before
# the next one), and the watchdog thread prints the line built so far when a
# design hangs.  SFL_BENCH_INJECT rehearses each failure (tests only):
#   fail:<design>[@<rank>]   run_design of <design> raises (on one rank or all)
#   hang:<design>[@<rank>]   run_design of <design> never returns
#   raise:rank<r>            rank r raises at start-up, before any collective
#   corrupt:<design>[@<rank>] the design's round-0 result check is off by one bit

def injected(kind: str, design: str | None, rank: int) -> bool:
    """Whether SFL_BENCH_INJECT asks for failure ``kind`` here (see above)."""
    spec = os.environ.get("SFL_BENCH_INJECT", "")
    for item in filter(None, spec.split(",")):
        k, _, rest = item.partition(":")
        if k != kind:
            continue
        if kind == "raise":
            if rest == f"rank{rank}":
                return True
            continue
        name, _, r = rest.partition("@")
        if name == design and (not r or int(r) == rank):
            return True
    return False


def inject_in_design(v_name: str, rank: int) -> None:
    if injected("fail", v_name, rank):
        raise RuntimeError(f"SFL_BENCH_INJECT: injected failure in design {v_name!r} on rank {rank}")
    if injected("hang", v_name, rank):
        print(f"bench.py rank {rank}: SFL_BENCH_INJECT: design {v_name!r} hangs", file=sys.stderr, flush=True)
        while True:
            time.sleep(3600)


class Watchdog:
    """Bounds a rank's run and keeps its measurement.

    * A design other than the headline that runs longer than
      ``variant_timeout`` seconds (or the run nearing ``total`` seconds after
      the headline finished) is declared hung: rank 0 prints the line built
      so far with that design marked and ``variants_incomplete``, every rank
      dumps its threads' stacks to stderr and exits 0 -- the headline stands.
    * Before the headline has finished there is nothing to keep: at
      ``total`` seconds ``faulthandler`` (a C thread, which fires even while
      the main thread holds the GIL) dumps every stack and exits 1.

    A Python thread, polled every 0.25 s: it runs while the main thread waits
    in a GIL-releasing call (a ctypes RCCL call, a device synchronise, a
    c10d wait), which is where a hung collective leaves it."""

    def __init__(self, total: float, variant_timeout: float, rank: int):
        import threading

        self.total, self.variant_timeout, self.rank = total, variant_timeout, rank
        self.t0 = time.monotonic()
        self.phase, self.t_phase = "setup", self.t0
        self.line = None        # rank 0's line so far, once the headline has finished
        self.pending = []       # designs not yet run
        self.lock = threading.Lock()
        self.printed = False
        if total > 0:
            import faulthandler

            faulthandler.dump_traceback_later(total, exit=True)
            threading.Thread(target=self._loop, name="bench-watchdog", daemon=True).start()

    def enter(self, phase: str) -> None:
        with self.lock:
            self.phase, self.t_phase = phase, time.monotonic()
            if phase in self.pending:
                self.pending.remove(phase)
        if os.environ.get("SFL_BENCH_TRACE"):  # phase timeline on stderr (the rehearsal tests set it)
            print(f"bench.py rank {self.rank}: phase {phase} at {self.t_phase - self.t0:.1f} s", file=sys.stderr,
                  flush=True)

    def emit(self, line: dict) -> bool:
        """Print ``line`` (rank 0), once per process."""
        with self.lock:
            if self.printed:
                return False
            self.printed = True
        print(json.dumps(line), flush=True)
        return True

    def _loop(self):
        warned = False
        while True:
            time.sleep(0.25)
            now = time.monotonic()
            with self.lock:
                phase, t_phase, line = self.phase, self.t_phase, self.line
            left = self.total - (now - self.t0)
            if line is not None and phase not in ("headline", "done") and (
                    now - t_phase > self.variant_timeout or left < 10):
                self._give_up(phase, now - t_phase)
            if line is None and left < 3 and not warned:
                warned = True
                print(f"bench.py rank {self.rank}: headline not finished after {self.total - 3:.0f} s; "
                      f"dumping every thread's stack and exiting", file=sys.stderr, flush=True)

    def _give_up(self, phase: str, waited: float):
        import copy
        import faulthandler

        with self.lock:
            line = copy.deepcopy(self.line)
            pending = list(self.pending)
        msg = (f"design {phase!r} did not finish within {waited:.0f} s on rank {self.rank} (hung); every rank's "
               f"stacks are on stderr; the headline and the designs before it stand")
        errs = published_errors(phase) if self.rank == 0 else []
        if errs:  # a rank that raised left its peers waiting in the design's collectives
            msg += "; errors raised by ranks: " + "; ".join(errs)
        print(f"bench.py rank {self.rank}: {msg}", file=sys.stderr, flush=True)
        if self.rank == 0 and phase == "check":  # the headline's result check hung: the designs after it never ran
            line["check"]["error"] = "hung"
            line["check"]["detail"] = msg
            line["variants_incomplete"] = True
            self.emit(line)
        elif self.rank == 0 and phase == "host_resident":  # after every design: only this field is lost
            line["host_resident"] = {"error": "hung", "detail": msg}
            self.emit(line)
        elif self.rank == 0:
            line.setdefault("exchange_variants", []).append({"name": phase, "error": "hung", "detail": msg})
            line["exchange_variants"] += [{"name": p, "error": "skipped", "detail": f"not run: {phase!r} hung"}
                                          for p in pending]
            line["variants_incomplete"] = True
            self.emit(line)
        faulthandler.dump_traceback(all_threads=True)
        sys.stderr.flush()
        os._exit(0)


def _store():
    """The process group's c10d store (torchrun's TCPStore): independent of
    the collectives, so a rank can leave a message there that rank 0 can read
    while a design's collectives hang."""
    try:
        import torch.distributed as dist

        if dist.is_initialized():
            return dist.distributed_c10d._get_default_store()
    except Exception:  # noqa: BLE001 -- best effort, the line does not depend on it
        pass
    return None


def publish_error(design: str, rank: int, text: str) -> None:
    s = _store()
    if s is not None:
        try:
            s.set(f"sfl_bench_err/{design}/{rank}", text)
        except Exception:  # noqa: BLE001
            pass


def published_errors(design: str, world: int | None = None) -> list[str]:
    s = _store()
    if s is None:
        return []
    world = world or int(os.environ.get("WORLD_SIZE", "1"))
    out = []
    for r in range(world):
        key = f"sfl_bench_err/{design}/{r}"
        try:
            if s.check([key]):
                out.append(s.get(key).decode(errors="replace"))
        except Exception:  # noqa: BLE001
            pass
    return out


def control_group(ctx):
    """A gloo group for agreement between designs: CPU tensors, so it still
    works when a design left the GPU streams or the RCCL communicator
    unusable."""
    import torch.distributed as dist

    if ctx.get("ctrl") is None:
        ctx["ctrl"] = dist.new_group(backend="gloo") if dist.get_backend() != "gloo" else dist.group.WORLD
    return ctx["ctrl"]


def run_variants(ctx, runner, variants, summarise, out: dict, wd: Watchdog, settle=None) -> None:
    """Every design after the headline, each contained: an exception on any
    rank is printed there (traceback on stderr) and recorded in its entry of
    out["exchange_variants"]; the ranks agree (gloo all_gather of the error
    texts) before the next design.  ``settle(ctx, result)`` (bench.py's
    combine_check) runs inside the containment, after the runner.  A design that failed on EVERY rank left
    no collective half-issued, so the next one runs; one that failed on some
    ranks only may have left the others' exchange pending, so the remaining
    designs are skipped and the line printed as it stands."""
    import traceback

    import torch.distributed as dist

    args, rank = ctx["args"], ctx["rank"]
    group = control_group(ctx)
    with wd.lock:
        wd.pending = [v.name for v in variants]
    for i, v in enumerate(variants):
        wd.enter(v.name)
        err = None
        try:
            res = runner(ctx, v, args.variant_steps, min(5, args.warmup))
            if settle is not None:
                settle(ctx, res)
        except Exception as e:  # noqa: BLE001 -- contained, reported in the line
            err = f"rank {rank}: {e!r}"
            print(f"bench.py rank {rank}: design {v.name!r} failed:", file=sys.stderr)
            traceback.print_exc()
            sys.stderr.flush()
            publish_error(v.name, rank, err)
        errs = [None] * ctx["world"]
        dist.all_gather_object(errs, err, group=group)
        failed = [e for e in errs if e is not None]
        with wd.lock:
            if not failed:
                entry = summarise(res)
                want = out.get("check", {}).get("decoded_digest")
                if want is not None and entry.get("check_digest") is not None and entry["check_digest"] != want:
                    entry["mismatch"] = f"round-0 result check {entry.get('check_digest')} != the headline's {want}"
                    out["designs_agree"] = False
                out["exchange_variants"].append(entry)
                continue
            out["exchange_variants"].append({"name": v.name, "error": "failed", "detail": "; ".join(failed)})
            if len(failed) < ctx["world"]:
                rest = [x.name for x in variants[i + 1:]]
                out["exchange_variants"] += [{"name": p, "error": "skipped",
                                              "detail": f"not run: {v.name!r} failed on some ranks only"}
                                             for p in rest]
                out["variants_incomplete"] = True
                wd.pending = []
                return
    with wd.lock:
        wd.pending = []


def run_contained(ctx, phase: str, fn, out: dict, wd: Watchdog) -> None:
    """One more measurement after the designs, contained like them: its
    result (or the ranks' errors) goes to out[phase]; a hang is the
    watchdog's (phase named)."""
    import traceback

    import torch.distributed as dist

    wd.enter(phase)
    err, res = None, None
    try:
        res = fn()
    except Exception as e:  # noqa: BLE001 -- contained, reported in the line
        err = f"rank {ctx['rank']}: {e!r}"
        traceback.print_exc()
        publish_error(phase, ctx["rank"], err)
    errs = [None] * ctx["world"]
    dist.all_gather_object(errs, err, group=control_group(ctx))
    failed = [e for e in errs if e is not None]
    with wd.lock:
        out[phase] = {"error": "failed", "detail": "; ".join(failed)} if failed else res


def variant_summary(x: dict) -> dict:
    return {"name": x["name"], "value": x["value"], "ms_per_step": x["ms_per_step"], "steps": x["steps"],
            "kernel_ms_per_step": x["kernel_ms_per_step"], "kernel": x["kernel"], "chunks": x["chunks"],
            "xchg_ms": x["exchange"]["ms_per_step"], "bytes_per_rank_per_step": x["exchange"]["bytes_per_rank_per_step"],
            "algbw_GBps": x["exchange"]["algbw_GBps"], "busbw_GBps": x["exchange"]["busbw_GBps"],
            "collective": x["exchange"]["collective"], "check_digest": x.get("check_digest"),
            "exchange_model": _model_brief(x["exchange"].get("model"))}


def _model_brief(m):
    """A design's exchange model in its variant entry (the full one is the
    headline's roofline.exchange)."""
    if not m:
        return None
    return {k: m[k] for k in ("bytes_per_link_per_step", "link_ms_at_peak", "link_frac", "predicted_ms_per_step",
                              "bound", "mode")}
