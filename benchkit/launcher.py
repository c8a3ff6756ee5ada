"""bench.py's self-launcher for ``--gpus N`` (no outer torchrun): the N rank
processes as one torch.distributed.run child, per-rank logs, and the
failing ranks' tracebacks printed after a failed run."""

from __future__ import annotations

import json
import os
import sys

from .baseline import cpu_baseline, rank_cpu_seconds


def launch_ranks(args, script: str) -> int:
    """`--gpus N` without an outer torchrun (WORLD_SIZE unset): measure the CPU
    baseline here, then start the N rank processes as ONE child process
    (torch.distributed.run with a c10d rendezvous on 127.0.0.1 port 0: the
    store binds a port the kernel picks, no probe-then-bind race) and return
    its exit code.  This process never touches the GPU (it imports no torch),
    so nothing is exec'd from a process that initialised HIP."""
    import subprocess
    import tempfile
    import uuid

    env = dict(os.environ)
    env.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
    if args.rehearse_one_gpu:
        # W rank processes on the one GPU plus a caller that holds a GPU
        # context of its own run slower (W + 1 > 8 processes on one GPU): say
        # so on stderr, the run itself is still valid
        holders = gpu_context_holders([os.getpid(), os.getppid()])
        if holders:
            sys.stderr.write(rehearsal_warning(holders, args.gpus) + "\n")
        # N ranks share one box's CPU quota (a 16-CPU cgroup on the test box,
        # throttled during rehearsals: DESIGN.md §5); a rank's host work is
        # small copies, so one OpenMP thread each, as torchrun's own default
        env["OMP_NUM_THREADS"] = "1"
    tmp = None
    if args.cpu_baseline_seconds > 0:
        cpu = cpu_baseline(args.clients, args.fxp_bits, rank_cpu_seconds(args, args.gpus),
                           parallel=args.gpus == 1 and not args.dry_run)
        fd, tmp = tempfile.mkstemp(prefix="sfl_bench_cpu_", suffix=".json")
        with os.fdopen(fd, "w") as f:
            json.dump(cpu, f)
        env["SFL_BENCH_CPU_BASELINE"] = tmp
    # every rank's stderr also goes to <log_dir>/.../<rank>/stderr.log (and
    # still to the console, prefixed by the rank), so a failing rank's
    # traceback survives the interleaving of eight ranks' output; stdout is
    # left alone (rank 0's JSON line stays a bare line)
    log_dir = tempfile.mkdtemp(prefix="sfl_bench_ranks_")
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes", "1", "--nproc-per-node", str(args.gpus),
           "--rdzv-backend", "c10d", "--rdzv-endpoint", "127.0.0.1:0", "--rdzv-id", f"sfl-bench-{uuid.uuid4().hex}",
           "--local-addr", "127.0.0.1", "--log-dir", log_dir, "--redirects", "2", "--tee", "2",
           os.path.abspath(script), *sys.argv[1:]]
    try:
        rc = subprocess.run(cmd, env=env).returncode
        if rc != 0:
            sys.stderr.write(failing_ranks_report(log_dir))
            sys.stderr.flush()
        return rc
    finally:
        if tmp:
            os.unlink(tmp)
        import shutil

        shutil.rmtree(log_dir, ignore_errors=True)


KFD = "/dev/kfd"


def gpu_context_holders(pids, device: str = KFD) -> list:
    """The processes among ``pids`` that have ``device`` open -- a process
    with a HIP context holds /dev/kfd -- read from /proc without touching
    the GPU (unreadable or vanished processes count as not holding it)."""
    out = []
    for pid in pids:
        try:
            fds = os.listdir(f"/proc/{pid}/fd")
        except OSError:
            continue
        for fd in fds:
            try:
                if os.readlink(f"/proc/{pid}/fd/{fd}") == device:
                    out.append(pid)
                    break
            except OSError:
                continue
    return out


def rehearsal_warning(holders, world: int) -> str:
    return (f"--rehearse-one-gpu: process(es) {holders} (this launcher or its caller) already hold a GPU context; "
            f"with {world} rank processes that puts {world + len(holders)} processes on the one GPU, where rehearsals "
            "run slower (W = 8 at 8 x 100M: 31 s instead of 9 s, profiles/r06/rehearsal_context_probe.txt); the "
            "driver's runs have one process per GPU.")


def failing_ranks_report(log_dir: str, lines_per_rank: int = 60) -> str:
    """After a failed torchrun child: for every rank whose error file or
    stderr log holds a traceback, its last traceback (torchrun's error.json
    from @record first, else the tail of stderr.log from the last
    'Traceback')."""
    import glob

    out = []
    for path in sorted(glob.glob(os.path.join(log_dir, "**", "stderr.log"), recursive=True)):
        rank_dir = os.path.dirname(path)
        rank = os.path.basename(rank_dir)
        text = ""
        err_json = os.path.join(rank_dir, "error.json")
        if os.path.exists(err_json):
            try:
                with open(err_json) as f:
                    msg = json.load(f).get("message", {})
                text = msg.get("extraInfo", {}).get("py_callstack", "") if isinstance(msg, dict) else str(msg)
            except (OSError, ValueError):
                text = ""
        if not text:
            with open(path, errors="replace") as f:
                log = f.read()
            # a Python exception, a fatal signal's stacks (faulthandler is
            # enabled in every rank) or the watchdog's stack dump at expiry
            i = max(log.rfind("Traceback (most recent call last)"), log.rfind("Fatal Python error"),
                    log.rfind("Timeout ("))
            if i < 0:
                continue
            text = log[i:]
        tail = text.rstrip().splitlines()[-lines_per_rank:]
        out.append(f"---- bench.py: rank {rank} failed; its last traceback ({os.path.relpath(path, log_dir)}) ----\n"
                   + "\n".join(tail) + "\n")
    if not out:
        return f"---- bench.py: the rank processes failed, no rank left a traceback under {log_dir} ----\n"
    return "".join(out)
