"""A secretflow stand-in with real party isolation -- test infrastructure.

secretflow itself is not installed, so the drop-in is
exercised against this: every party is a SPAWNED process, ``pyu(fn,
num_returns=k)(*args)`` ships ``fn`` (cloudpickle, as Ray does) and runs it
there, and the driver only ever holds opaque handles.  Like secretflow:

* device objects in the arguments (nested in lists / tuples / dicts too)
  resolve to their values inside the party; an object of another party is
  refused (secretflow requires ``.to()`` first);
* ``obj.to(dev)`` moves the value between party processes; the driver relays
  the pickled bytes without unpickling them (Ray's object store role);
* ``reveal(obj)`` brings a value to the driver -- and here it RAISES for any
  value owned by a party in ``private`` that is not a plain ``int`` (the DH
  public keys are the only client values the protocol reveals), so a test
  passing through it proves no client datum, masked vector or generator
  state reached the driver.

``Cluster(..., lazy=True)`` defers a failing call's error to where its
results are used (``reveal``, an argument of a later call), as Ray does.

``make_package(cluster)`` builds fake ``secretflow``, ``secretflow.security``
and ``secretflow.security.aggregation`` modules whose ``SecureAggregator`` is
a placeholder, for ``install()`` tests.
"""
from __future__ import annotations

import itertools
import multiprocessing as mp
import pickle
import sys
import traceback
import types
from dataclasses import dataclass


class RevealRefused(PermissionError):
    """The driver asked for a client-owned value that is not public."""


class RemoteError(RuntimeError):
    """An exception inside a party process (its traceback is the message)."""


@dataclass(frozen=True)
class Handle:
    party: str
    oid: int


@dataclass(frozen=True)
class _Failed:
    """A lazy cluster's result of a call that raised: stored in place of the
    results, raised again wherever it is used (Ray's error propagation)."""
    name: str
    tb: str


class UpstreamError(RuntimeError):
    """A lazy cluster's object whose producing call failed."""


def _check(v):
    if isinstance(v, _Failed):
        raise UpstreamError(f"{v.name} upstream:\n{v.tb}")
    return v


def _resolve(x, party, store):
    if isinstance(x, Handle):
        if x.party != party:
            raise ValueError(f"object of {x.party} used on {party}; move it with .to() first")
        return _check(store[x.oid])
    if isinstance(x, (list, tuple)):
        return type(x)(_resolve(v, party, store) for v in x)
    if isinstance(x, dict):
        return {k: _resolve(v, party, store) for k, v in x.items()}
    return x


def _worker_main(party, conn, init, private, lazy=False):
    import cloudpickle

    if init is not None:
        cloudpickle.loads(init)()
    store, ids = {}, itertools.count()
    while True:
        op, args = conn.recv()
        if op == "stop":
            conn.send((True, None))
            return
        try:
            if op == "run":
                fn_b, call_b, num_returns = args
                fn = cloudpickle.loads(fn_b)
                try:
                    a, k = _resolve(cloudpickle.loads(call_b), party, store)
                    out = fn(*a, **k)
                    outs = list(out) if num_returns and num_returns > 1 else [out]
                    if num_returns and num_returns > 1 and len(outs) != num_returns:
                        raise ValueError(f"{fn} returned {len(outs)} values, num_returns={num_returns}")
                except Exception as e:  # noqa: BLE001
                    if not lazy:
                        raise
                    # lazy: the call "succeeds" with failed results; the error
                    # surfaces where they are used
                    f = _Failed(type(e).__name__, "".join(traceback.format_exception(e)))
                    outs = [f] * (num_returns if num_returns and num_returns > 1 else 1)
                oids = []
                for o in outs:
                    oid = next(ids)
                    store[oid] = o
                    oids.append(oid)
                res = oids
            elif op == "get":
                res = pickle.dumps(store[args[0]])
            elif op == "put":
                oid = next(ids)
                store[oid] = pickle.loads(args[0])
                res = oid
            elif op == "reveal":
                v = _check(store[args[0]])
                if private and not (isinstance(v, int) and not isinstance(v, bool)):
                    raise RevealRefused(f"reveal of a {type(v).__name__} owned by client {party}")
                res = pickle.dumps(v)
            elif op == "types":  # test hook: type names of everything held here
                res = sorted({type(v).__name__ for v in store.values()})
            else:
                raise ValueError(op)
            conn.send((True, res))
        except BaseException as e:  # noqa: BLE001 - reported to the driver
            conn.send((False, (type(e).__name__, "".join(traceback.format_exception(e)))))


class Cluster:
    """One spawned process per party.  ``private``: the client parties whose
    values ``reveal`` refuses (all but public ints).  ``init``: a callable
    each process runs first (cloudpickled)."""

    def __init__(self, parties, private=(), init=None, lazy=False):
        import cloudpickle

        ctx = mp.get_context("spawn")
        self.workers = {}
        ib = cloudpickle.dumps(init) if init is not None else None
        for p in parties:
            parent, child = ctx.Pipe()
            proc = ctx.Process(target=_worker_main, args=(p, child, ib, p in set(private), lazy), daemon=True)
            proc.start()
            self.workers[p] = (proc, parent)
        self.reveals = []  # (party, type) of every successful reveal

    def call(self, party, op, *args):
        proc, conn = self.workers[party]
        conn.send((op, args))
        ok, res = conn.recv()
        if not ok:
            name, tb = res
            if name == "RevealRefused":
                raise RevealRefused(tb.strip().splitlines()[-1])
            raise RemoteError(f"{name} in party {party}:\n{tb}")
        return res

    def pyu(self, party):
        return PYU(self, party)

    def close(self):
        for p, (proc, conn) in self.workers.items():
            try:
                conn.send(("stop", ()))
                conn.recv()
            except (OSError, EOFError):
                pass
            proc.join(timeout=30)
            if proc.is_alive():
                proc.kill()
        self.workers = {}

    def types_held(self, party):
        return self.call(party, "types")


class PYU:
    """secretflow.PYU shape: ``.party``; ``pyu(fn, num_returns=k)(*args)``."""

    def __init__(self, cluster: Cluster, party: str):
        self.cluster = cluster
        self.party = party

    def __call__(self, fn, num_returns=None, **_kw):
        import cloudpickle

        def run(*args, **kwargs):
            call = cloudpickle.dumps(_to_handles((args, kwargs), self))
            oids = self.cluster.call(self.party, "run", cloudpickle.dumps(fn), call, num_returns)
            objs = [PYUObject(self, oid) for oid in oids]
            return objs if num_returns and num_returns > 1 else objs[0]

        return run

    def __eq__(self, other):
        return isinstance(other, PYU) and other.party == self.party

    def __hash__(self):
        return hash(("PYU", self.party))

    def __repr__(self):
        return f"PYU({self.party})"


class PYUObject:
    """secretflow.PYUObject shape: ``.device`` and an opaque reference."""

    def __init__(self, device: PYU, oid: int):
        self.device = device
        self._oid = oid

    @property
    def handle(self):
        return Handle(self.device.party, self._oid)

    def to(self, device: PYU) -> "PYUObject":
        c = self.device.cluster
        blob = c.call(self.device.party, "get", self._oid)  # relayed, never unpickled here
        return PYUObject(device, c.call(device.party, "put", blob))

    def __repr__(self):
        return f"PYUObject({self.device.party}#{self._oid})"


def _to_handles(x, dev):
    if isinstance(x, PYUObject):
        return x.handle
    if isinstance(x, (list, tuple)):
        return type(x)(_to_handles(v, dev) for v in x)
    if isinstance(x, dict):
        return {k: _to_handles(v, dev) for k, v in x.items()}
    return x


def reveal(obj):
    if isinstance(obj, (list, tuple)):
        return type(obj)(reveal(o) for o in obj)
    if isinstance(obj, dict):
        return {k: reveal(v) for k, v in obj.items()}
    if isinstance(obj, PYUObject):
        c = obj.device.cluster
        v = pickle.loads(c.call(obj.device.party, "reveal", obj._oid))
        c.reveals.append((obj.device.party, type(v).__name__))
        return v
    return obj


class _PlaceholderSecureAggregator:
    """secretflow's own class (not installed): using it is an error."""

    def __init__(self, *a, **k):
        raise RuntimeError("secretflow's SecureAggregator is not available here; install() the HIP one")


def make_package():
    """Fake ``secretflow`` / ``.security`` / ``.security.aggregation`` modules
    (to be put into ``sys.modules`` by the caller)."""
    sf = types.ModuleType("secretflow")
    sf.__path__ = []
    sec = types.ModuleType("secretflow.security")
    sec.__path__ = []
    agg = types.ModuleType("secretflow.security.aggregation")
    agg.__path__ = []
    sf.PYU, sf.PYUObject, sf.DeviceObject, sf.reveal = PYU, PYUObject, PYUObject, reveal
    # a fresh class per package: subclasses made in one test do not leak into the next
    placeholder = type("SecureAggregator", (_PlaceholderSecureAggregator,), {})
    agg.SecureAggregator = placeholder
    sec.SecureAggregator = placeholder
    sec.aggregation = agg
    sf.security = sec
    return {"secretflow": sf, "secretflow.security": sec, "secretflow.security.aggregation": agg}


def installed_into(monkeypatch):
    """Put the fake package into ``sys.modules`` for one test."""
    mods = make_package()
    for name, m in mods.items():
        monkeypatch.setitem(sys.modules, name, m)
    return mods
