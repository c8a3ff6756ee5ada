"""RCCL's own account of an N > 1 run, for the bench line's ``rccl`` record.

Every rank of ``bench.py --gpus N`` (N > 1) writes RCCL's init log to a file
of its own (``NCCL_DEBUG=INFO``, ``NCCL_DEBUG_SUBSYS=INIT,P2P,SHM,NET``,
``NCCL_DEBUG_FILE``) -- a file, so rank 0's stdout stays one JSON line.
After the headline, each rank parses its file (``summarise``) and rank 0
gathers the summaries: which transport RCCL chose per connection (P2P/IPC
over xGMI on the node, SHM, or NET/Socket -- what the one-GPU rehearsal's
NCCL_HOSTID trick gives), how many ranks and nodes it saw, together with
``ncclCommCount`` / ``ncclCommCuDevice`` from the library (``sa_comm_info``).
The first 8-GPU record then shows by itself whether xGMI carried the
exchange.  Replaces nothing in the reference (its exchange is RayFed's
object store, ``sfl/distributed/op_strategy.py:131-141``); it audits ours.
"""

from __future__ import annotations

import glob
import os
import re

# the variables only the one-GPU rehearsal may set (benchkit/standin.py
# one_gpu_rccl_env): each one would push the node's exchange off xGMI
REHEARSAL_ONLY_ENV = ("NCCL_HOSTID", "NCCL_SOCKET_IFNAME", "NCCL_IB_DISABLE")

_NRANKS = re.compile(r"\bn[Rr]anks (\d+)")
_NNODES = re.compile(r"\bnNodes (\d+)")


def debug_env(rank: int, log_dir: str) -> dict:
    """The environment that sends this rank's RCCL init log to
    ``<log_dir>/rank<r>.<pid>.log`` (RCCL expands %p).  Empty when the caller
    already routes RCCL's log somewhere (NCCL_DEBUG_FILE set): we do not take
    it over, and the record then says so."""
    if os.environ.get("NCCL_DEBUG_FILE"):
        return {}
    # INFO at least (the GPU box exports NCCL_DEBUG=VERSION, which logs no
    # connection); it goes to the file, so the console stays as it was
    level = os.environ.get("NCCL_DEBUG", "").upper()
    return {"NCCL_DEBUG": level if level in ("INFO", "TRACE") else "INFO",
            "NCCL_DEBUG_SUBSYS": "INIT,P2P,SHM,NET",
            "NCCL_DEBUG_FILE": os.path.join(log_dir, f"rank{rank}.%p.log")}


def transport_of(line: str) -> str | None:
    """The transport family of one RCCL connection line, e.g.
    ``... Channel 00/0 : 0[0] -> 1[1] via P2P/IPC/read`` -> ``P2P/IPC``,
    ``... [send] via NET/Socket/0`` -> ``NET/Socket``, ``via SHM/direct/direct``
    -> ``SHM/direct``, ``via P2P/direct pointer/read`` -> ``P2P/direct pointer``;
    None for any other line."""
    if " via " not in line or "Channel" not in line:
        return None
    tail = line.split(" via ", 1)[1].strip()
    words = []
    for w in tail.split():
        if w == "comm" or w.startswith("0x") or w.startswith("["):
            break
        words.append(w)
    parts = " ".join(words).split("/")
    if not parts or not parts[0]:
        return None
    return "/".join(p.strip() for p in parts[:2])


def summarise(text: str) -> dict:
    """One rank's log -> {"transports": {family: connections}, "nranks": [...],
    "nnodes": [...], "lines": n}.  ``nranks`` / ``nnodes`` are every value the
    init lines state (one per communicator: torch's process group and ours)."""
    transports: dict[str, int] = {}
    nranks, nnodes = set(), set()
    lines = 0
    for line in text.splitlines():
        if "NCCL INFO" not in line:
            continue
        lines += 1
        t = transport_of(line)
        if t:
            transports[t] = transports.get(t, 0) + 1
        m = _NRANKS.search(line)
        if m:
            nranks.add(int(m.group(1)))
        m = _NNODES.search(line)
        if m:
            nnodes.add(int(m.group(1)))
    return {"transports": transports, "nranks": sorted(nranks), "nnodes": sorted(nnodes), "lines": lines}


def rank_summary(rank: int, log_dir: str | None, comm_info: dict | None) -> dict:
    """This rank's record: its parsed log file(s) plus ``sa_comm_info``."""
    out = {"rank": rank, "comm": comm_info}
    if log_dir is None:
        out["log"] = None
        out["note"] = "NCCL_DEBUG_FILE was set by the caller: RCCL's log not taken over"
        return out
    text = ""
    for f in sorted(glob.glob(os.path.join(log_dir, f"rank{rank}.*.log"))):
        with open(f, errors="replace") as fh:
            text += fh.read()
    out["log"] = summarise(text)
    return out


def combine(per_rank: list, world: int) -> dict:
    """Rank 0's ``rccl`` record from every rank's summary: the transport
    families summed over ranks (connections), the rank / node counts RCCL
    stated, and ``xgmi``: True iff every connection RCCL logged is P2P (IPC
    or direct) -- the peer-to-peer path over xGMI on one node; False if any
    went over SHM or the network; None if nothing was logged."""
    transports: dict[str, int] = {}
    nranks, nnodes, devices, lines = set(), set(), [], 0
    for r in per_rank:
        log = r.get("log") or {}
        for k, v in log.get("transports", {}).items():
            transports[k] = transports.get(k, 0) + v
        nranks.update(log.get("nranks", []))
        nnodes.update(log.get("nnodes", []))
        lines += log.get("lines", 0)
        devices.append((r.get("comm") or {}).get("device"))
    xgmi = None
    if transports:
        xgmi = all(k.startswith("P2P") for k in transports)
    comm_nranks = sorted({(r.get("comm") or {}).get("nranks") for r in per_rank} - {None})
    return {"world": world, "nranks": comm_nranks[0] if len(comm_nranks) == 1 else comm_nranks,
            "nranks_logged": sorted(nranks), "nnodes_logged": sorted(nnodes),
            "devices": devices, "transports": transports, "xgmi": xgmi, "log_lines": lines,
            "rehearsal_env": {k: os.environ[k] for k in REHEARSAL_ONLY_ENV if k in os.environ},
            "source": "per-rank RCCL init logs (NCCL_DEBUG=INFO, SUBSYS INIT,P2P,SHM,NET, NCCL_DEBUG_FILE) "
                      "and ncclCommCount / ncclCommCuDevice (sa_comm_info)"}
