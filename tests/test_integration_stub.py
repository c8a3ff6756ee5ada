"""INTEGRATION.md's reference-side glue is code a maintainer copies: run it.

The ctypes stub (§2) and the party-side ``mask()`` with numpy's rejection
re-draw (§3) are extracted from the document and executed as written, on a
PCG64 stream whose raw draw at a chosen element is 0.  numpy's own
``Generator.integers(int64.min, int64.max)`` (the reference's mask draw)
rejects that draw; the stub's masked vector and stream position must match
it bit for bit, over two calls."""
import os
import re

import numpy as np
import pytest

torch = pytest.importorskip("torch")
pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _blocks():
    text = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    return re.findall(r"```python\n(.*?)```", text, re.S)


def _stub_namespace():
    blocks = _blocks()
    stub = next(b for b in blocks if "class PCG64(C.Structure)" in b)
    party = next(b for b in blocks if "def mask(self, datum, weight=1):" in b)
    redraw = next(b for b in blocks if "lib.sa_stream_shift.argtypes" in b)
    ns = {"__file__": os.path.join(ROOT, "sfl_amd", "lib", "sfl_sa.py")}
    exec(compile(stub, "INTEGRATION.md#2", "exec"), ns)
    exec(compile(redraw, "INTEGRATION.md#3-bindings", "exec"), ns)
    exec(compile(party, "INTEGRATION.md#3", "exec"), ns)
    return ns


def _state_with_zero_at(e):
    from oracle import secagg as o

    A, M, inc = o.PCG64_MULT, (1 << 128) - 1, (98765 << 1) | 1
    target = (0x0123456789ABCDEF << 64) | 0x0123456789ABCDEF  # hi == lo: XSL-RR output 0
    ainv = pow(A, -1, 1 << 128)
    s = ((target - inc) * ainv) & M  # the state whose step yields the 0
    for _ in range(e):
        s = ((s - inc) * ainv) & M
    assert o.pcg64_raw_py(s, inc, e + 1)[e] == 0
    return s, inc


def test_integration_stub_mask_reproduces_numpy_rejection():
    if not torch.cuda.is_available():
        pytest.skip("no GPU")
    from oracle import secagg as o

    ns = _stub_namespace()
    U128, PCG64 = ns["U128"], ns["PCG64"]
    s, inc = _state_with_zero_at(1000)

    class Party:
        mask, _redraw = ns["mask"], ns["_redraw"]

        def __init__(self):
            self.party, self.peers, self.fxp_bits = "alice", ["bob"], 18
            self.gens = {"bob": PCG64(U128(s & (2**64 - 1), s >> 64), U128(inc & (2**64 - 1), inc >> 64))}
            self.pos = {"bob": 0}

    bg = np.random.PCG64()
    bg.state = {"bit_generator": "PCG64", "state": {"state": s, "inc": inc}, "has_uint32": 0, "uinteger": 0}
    gen = np.random.Generator(bg)
    p = Party()
    rng = np.random.default_rng(3)
    for n in (4099, 3001):  # the zero lands in the first call; the second checks the shifted position
        x = (rng.standard_normal(n) * 1e-2).astype(np.float32)
        got = p.mask(x).cpu().numpy().view(np.uint64)
        m = gen.integers(o.INT64_MIN, o.INT64_MAX, size=n).astype(np.uint64)
        assert np.array_equal(got, o.quantize(x) + m)  # bob sorts after alice: +m
    assert p.pos["bob"] == 4099 + 3001 + 1  # numpy consumed one raw draw more
