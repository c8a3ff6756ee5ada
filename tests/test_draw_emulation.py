"""The generated PCG64 draw asm (sfl_amd/csrc/sa_draw2.h), executed on the CPU.

A small interpreter runs every pair-draw variant's asm block instruction by
instruction on one lane -- each opcode's gfx950 semantics, carries in SGPR
bits, 64-bit VGPR pairs, and the state pair's halves aliased the way the
build-checked ISA places them (tools/check_pair01.py) -- and the result is
compared with numpy's PCG64 (the reference's PRG): the next states, the
accumulated masks of both clients (added, or subtracted), and the raw == 0
running minimum.  Inputs include rotations r = 0, r < 32, r >= 32 and a raw
draw of 0, so both rotation forms the generator can emit are pinned here
before any GPU runs them."""
import os
import re

import numpy as np
import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
M32, M64, M128 = (1 << 32) - 1, (1 << 64) - 1, (1 << 128) - 1
A = 0x2360ED051FC65DA44385DF649FCCF645

# %[name] operands that are 64-bit values (VGPR pairs or SGPR pairs)
WIDE = {"p01a", "p01b", "ua", "ub", "va", "vb", "bua", "bub", "bva", "bvb",
        "c0a", "c1a", "c23a", "c0b", "c1b", "c23b", "mma", "mmb",
        "u", "v", "mm", "c0", "c1", "c23"}  # the last six: the single draw (sa_clients_impl.h)


def _functions(text):
    """name -> {F: asm lines} of every generated draw function."""
    out = {}
    for m in re.finditer(r"void (pcg_draw2_\w+)\((.*?)\n}\n", text, re.S):
        name, body = m.group(1), m.group(2)
        blocks = {}
        for fm in re.finditer(r"F == (\d+)\) \{\n    asm volatile\(\n(.*?)\n        :", body, re.S):
            blocks[int(fm.group(1))] = re.findall(r'"(.*?)\\n\\t"', fm.group(2))
        out[name] = blocks
    return out


class Lane:
    def __init__(self, env, rng):
        # the draw's scratch VGPRs start as junk: results must not depend on it
        self.v = {i: int(rng.integers(0, 1 << 32)) for i in range(20)}
        self.env = env  # bound %[operands]

    # operand access --------------------------------------------------------
    def read(self, op, wide=False):
        op = op.strip()
        m = re.fullmatch(r"v\[(\d+):(\d+)\]", op)
        if m:
            lo, hi = int(m.group(1)), int(m.group(2))
            assert hi == lo + 1
            return self.v[lo] | (self.v[hi] << 32)
        m = re.fullmatch(r"v(\d+)", op)
        if m:
            return self.v[int(m.group(1))]
        m = re.fullmatch(r"%\[(\w+)\]", op)
        if m:
            n = m.group(1)
            if n in ("s0a", "s1a", "s0b", "s1b"):  # halves of the state pair p01 (the ISA-checked alias)
                p = self.env["p01" + n[2]]
                return p & M32 if n[1] == "0" else p >> 32
            if n.endswith("lo") or n.endswith("hi"):
                return self.env[n]
            return self.env[n]
        if op == "vcc":
            return self.env["vcc"]
        return int(op, 0)

    def write(self, op, val):
        op = op.strip()
        m = re.fullmatch(r"v\[(\d+):(\d+)\]", op)
        if m:
            lo = int(m.group(1))
            self.v[lo], self.v[lo + 1] = val & M32, (val >> 32) & M32
            return
        m = re.fullmatch(r"v(\d+)", op)
        if m:
            self.v[int(m.group(1))] = val & M32
            return
        m = re.fullmatch(r"%\[(\w+)\]", op)
        if m:
            n = m.group(1)
            if n in ("s0a", "s1a", "s0b", "s1b"):
                k = "p01" + n[2]
                p = self.env[k]
                self.env[k] = (p & ~M32 & M64) | (val & M32) if n[1] == "0" else (p & M32) | ((val & M32) << 32)
                return
            self.env[n] = val & (M64 if n in WIDE else M32) if not n.startswith("k") and n not in ("swb",) else val
            return
        if op == "vcc":
            self.env["vcc"] = val
            return
        raise ValueError(op)

    # one instruction -------------------------------------------------------
    def run(self, line):
        line = line.strip()
        if line.startswith("s_nop"):
            return
        lut = None
        m = re.search(r"\s+bitop3:(0x[0-9a-f]+)$", line)
        if m:
            lut = int(m.group(1), 16)
            line = line[:m.start()]
        opc, rest = line.split(None, 1)
        ops = [o.strip() for o in rest.split(",")]
        r = self.read
        if opc == "v_mad_u64_u32":
            t = r(ops[2]) * r(ops[3]) + r(ops[4])
            self.write(ops[0], t & M64)
            self.write(ops[1], t >> 64)
        elif opc == "v_mul_lo_u32":
            self.write(ops[0], r(ops[1]) * r(ops[2]))
        elif opc == "v_add_co_u32_e64":
            t = r(ops[2]) + r(ops[3])
            self.write(ops[0], t)
            self.write(ops[1], t >> 32)
        elif opc == "v_addc_co_u32_e64":
            t = r(ops[2]) + r(ops[3]) + (r(ops[4]) & 1)
            self.write(ops[0], t)
            self.write(ops[1], t >> 32)
        elif opc == "v_sub_co_u32_e64":
            t = r(ops[2]) - r(ops[3])
            self.write(ops[0], t & M32)
            self.write(ops[1], 1 if t < 0 else 0)
        elif opc == "v_subb_co_u32_e64":
            t = r(ops[2]) - r(ops[3]) - (r(ops[4]) & 1)
            self.write(ops[0], t & M32)
            self.write(ops[1], 1 if t < 0 else 0)
        elif opc == "v_bitop3_b32":
            a, b, c = r(ops[1]), r(ops[2]), r(ops[3])
            out = 0
            for i in range(32):
                idx = ((a >> i) & 1) << 2 | ((b >> i) & 1) << 1 | ((c >> i) & 1)
                out |= ((lut >> idx) & 1) << i
            self.write(ops[0], out)
        elif opc == "v_lshrrev_b32_e32":
            self.write(ops[0], r(ops[2]) >> (r(ops[1]) & 31))
        elif opc == "v_sub_u32_e32":
            self.write(ops[0], r(ops[1]) - r(ops[2]))
        elif opc == "v_lshrrev_b64":
            self.write(ops[0], r(ops[2]) >> (r(ops[1]) & 63))
        elif opc == "v_lshlrev_b64":
            self.write(ops[0], (r(ops[2]) << (r(ops[1]) & 63)) & M64)
        elif opc in ("v_or_b32_e32", "v_or_b32"):
            self.write(ops[0], r(ops[1]) | r(ops[2]))
        elif opc == "v_mov_b32_e32":
            self.write(ops[0], r(ops[1]))
        elif opc == "v_xor_b32_e32":
            self.write(ops[0], r(ops[1]) ^ r(ops[2]))
        elif opc in ("v_cmp_eq_u64_e32", "v_cmp_eq_u64_e64"):
            # this lane's bit of the compare mask (one lane: bit 0)
            self.write(ops[0], 1 if r(ops[1]) == r(ops[2]) else 0)
        elif opc == "s_or_b64":
            self.write(ops[0], r(ops[1]) | r(ops[2]))
        elif opc == "v_min3_u32":
            self.write(ops[0], min(r(ops[1]), r(ops[2]), r(ops[3])))
        elif opc == "v_lshl_add_u64":
            self.write(ops[0], ((r(ops[1]) << r(ops[2])) + r(ops[3])) & M64)
        elif opc == "v_alignbit_b32":
            self.write(ops[0], ((r(ops[1]) << 32 | r(ops[2])) >> (r(ops[3]) & 31)) & M32)
        elif opc in ("v_cmp_gt_i32_e32", "v_cmp_gt_i32_e64"):
            x = r(ops[2])
            self.write(ops[0], 1 if (x - (1 << 32) if x >> 31 else x) < 0 else 0)
        elif opc in ("v_cndmask_b32_e32", "v_cndmask_b32_e64"):
            self.write(ops[0], r(ops[2]) if r(ops[3]) & 1 else r(ops[1]))
        else:
            raise NotImplementedError(opc)


def _raw(s):
    hi, lo = s >> 64, s & M64
    x, rot = hi ^ lo, hi >> 58
    return ((x >> rot) | (x << (64 - rot))) & M64


def _states(rng):
    """Start states (before the step) whose next state rotates by r = 0, a
    small r, a large r, and one that draws raw 0."""
    inc = (int(rng.integers(1, 1 << 62)) << 66 | int(rng.integers(0, 1 << 62))) | 1
    inc &= M128
    ainv = pow(A, -1, 1 << 128)
    out = []
    for want in ("r0", "small", "large", "zero", "rand", "rand"):
        while True:
            if want == "zero":
                w = int(rng.integers(0, 1 << 62))
                nxt = (w << 64) | w
            else:
                nxt = int(rng.integers(0, 1 << 63)) << 65 | int(rng.integers(0, 1 << 63)) << 2 | 3
                nxt &= M128
                if want == "r0":
                    nxt &= ~(0x3F << 122) & M128
                elif want == "small":
                    nxt = (nxt & ~(0x3F << 122)) | (5 << 122)
                elif want == "large":
                    nxt = (nxt & ~(0x3F << 122)) | (45 << 122)
            s = ((nxt - inc) * ainv) & M128
            break
        out.append((s, inc))
    return out


def _check(fn_lines, kind, sa, sb, ma, mb, acc, rng):
    ia, ib = sa[1], sb[1]
    a_limbs = [(A >> (32 * i)) & M32 for i in range(4)]
    env = {"a0": a_limbs[0], "a1": a_limbs[1], "a2": a_limbs[2], "a3": a_limbs[3],
           "ma": ma, "mb": mb, "mma": ma << 32 | ma, "mmb": mb << 32 | mb, "zmin": M32, "zh": 0}
    for t, (s, inc) in (("a", sa), ("b", sb)):
        env[f"p01{t}"] = s & M64
        env[f"s2{t}"] = (s >> 64) & M32
        env[f"s3{t}"] = s >> 96
        env[f"c0{t}"] = inc & M32
        env[f"c1{t}"] = (inc >> 32) & M32
        env[f"c23{t}"] = inc >> 64
    env.update(acc)
    for k in ("va", "vb"):  # the subtracting partners' halves
        if k in acc:
            env[k + "lo"], env[k + "hi"] = acc[k] & M32, acc[k] >> 32
    lane = Lane(env, rng)
    for line in fn_lines:
        lane.run(line)
    # expected
    exp_state, t = {}, {}
    zero = False
    for tag, (s, inc), m in (("a", sa, ma), ("b", sb, mb)):
        nxt = (s * A + inc) & M128
        exp_state[tag] = nxt
        raw = _raw(nxt)
        zero |= raw == 0
        t[tag] = raw ^ (M64 if m else 0)
    for tag in "ab":
        got = lane.env[f"p01{tag}"] | lane.env[f"s2{tag}"] << 64 | lane.env[f"s3{tag}"] << 96
        assert got == exp_state[tag], (kind, tag)
    if any("%[zh]" in ln for ln in fn_lines):  # shift-rotation form: SALU-OR-ed 64-bit compares
        assert (lane.env["zh"] != 0) == zero, kind
    else:  # alignbit / rot64 forms: the per-lane running minimum
        assert (lane.env["zmin"] == 0) == zero, kind
    return lane.env, t


@pytest.mark.parametrize("variant", ["ss", "sa", "as", "aa"])
def test_pair_draw_blocks_equal_numpy_pcg64(variant):
    funcs = _functions(open(os.path.join(ROOT, "sfl_amd", "csrc", "sa_draw2.h")).read())
    lines = funcs[f"pcg_draw2_pair_{variant}"][0]
    rng = np.random.default_rng(sum(map(ord, variant)))
    states = _states(rng)
    checked = 0
    for i, sa in enumerate(states):
        sb = states[(i + 3) % len(states)]
        for ma, mb in ((0, 0), (M32, 0), (0, M32), (M32, M32)):
            acc = {k: int(rng.integers(0, 1 << 63)) * 2 + 1 for k in ("ua", "ub", "va", "vb")}
            env, t = _check(lines, variant, sa, sb, ma, mb, acc, rng)
            assert env["ua"] == (acc["ua"] + t["a"]) & M64
            assert env["ub"] == (acc["ub"] + t["b"]) & M64
            for tag, mode in zip("ab", variant):
                k = "v" + tag
                got = env[k] if mode == "a" else env[k + "lo"] | env[k + "hi"] << 32
                want = (acc[k] + t[tag]) & M64 if mode == "a" else (acc[k] - t[tag]) & M64
                assert got == want, (variant, tag, mode)
            checked += 1
    assert checked == 24


@pytest.mark.parametrize("name", ["pcg_draw2_one", "pcg_draw2_one_same"])
def test_one_sided_draw_blocks_equal_numpy_pcg64(name):
    funcs = _functions(open(os.path.join(ROOT, "sfl_amd", "csrc", "sa_draw2.h")).read())
    lines = funcs[name][0]
    rng = np.random.default_rng(len(name))
    states = _states(rng)
    for i, sa in enumerate(states):
        sb = states[(i + 1) % len(states)]
        for ma, mb in ((0, 0), (M32, M32), (0, M32)):
            acc = {k: int(rng.integers(0, 1 << 63)) for k in ("ua", "ub")}
            env, t = _check(lines, name, sa, sb, ma, mb, acc, rng)
            if name.endswith("same"):  # both cross streams of one client
                assert env["ua"] == (acc["ua"] + t["a"] + t["b"]) & M64
            else:
                assert env["ua"] == (acc["ua"] + t["a"]) & M64
                assert env["ub"] == (acc["ub"] + t["b"]) & M64


@pytest.mark.parametrize("flag", ["--alignbit", "--rot64", "--zmin"])
def test_other_rotation_forms_of_the_generator(flag):
    """The committed header carries the shift-rotation form (the generator's
    default: two 64-bit shifts joined by one v_lshl_add_u64, the raw == 0 test
    as a 64-bit compare OR-ed on the SALU); the generator's --alignbit form
    (round 2: two v_alignbit + a swap on bit 31) and --rot64 form (shifts +
    OR) compute the same draws."""
    import subprocess
    import sys

    text = open(os.path.join(ROOT, "sfl_amd", "csrc", "sa_draw2.h")).read()
    assert "v_lshl_add_u64 v[6:7], v[6:7], 1, v[4:5]" in text and "v_alignbit_b32" not in text
    assert '#define SA_DRAW2_FORM "rots"' in text
    alt = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_draw2.py"), flag],
                         capture_output=True, text=True, check=True).stdout
    assert ("v_alignbit_b32" in alt) == (flag == "--alignbit") and "v_cmp_eq_u64" not in alt
    funcs = _functions(alt)
    rng = np.random.default_rng(64)
    states = _states(rng)
    for variant in ("ss", "sa", "as", "aa"):
        lines = funcs[f"pcg_draw2_pair_{variant}"][0]
        for i, sa in enumerate(states):
            acc = {k: int(rng.integers(0, 1 << 63)) for k in ("ua", "ub", "va", "vb")}
            env, t = _check(lines, variant, sa, states[i - 1], M32 * (i & 1), 0, acc, rng)
            assert env["ua"] == (acc["ua"] + t["a"]) & M64


def _single_draw_functions():
    """name -> asm lines of the single-draw functions of sa_clients_impl.h
    (the SA_PCG_DRAW_ASM macro + each function's own accumulate tail)."""
    text = open(os.path.join(ROOT, "sfl_amd", "csrc", "sa_clients_impl.h")).read()
    mac = text[text.index("#define SA_PCG_DRAW_ASM"):text.index("#define SA_PCG_DRAW_OUTS")]
    head = re.findall(r'"(.*?)\\n\\t"', mac)
    out = {}
    for name in ("pcg_draw_pair", "pcg_draw_pair_a", "pcg_draw_one"):
        m = re.search(r"void " + name + r"\(.*?asm volatile\(SA_PCG_DRAW_ASM(.*?)\n\s*:", text, re.S)
        tail = [t.replace("\\n\\t", "") for t in re.findall(r'"(.*?)"', m.group(1))]
        out[name] = head + tail
    return out


@pytest.mark.parametrize("name", ["pcg_draw_pair", "pcg_draw_pair_a", "pcg_draw_one"])
def test_single_draw_equals_numpy_pcg64(name):
    """The single draws (odd leftover streams) in the same shift-rotation form:
    next state, accumulators (u adds; the partner subtracts, or adds when the
    kernel keeps it negated) and the SGPR raw == 0 mask, vs numpy's PCG64."""
    lines = _single_draw_functions()[name]
    assert any("v_lshl_add_u64 v[6:7], v[6:7], 1, v[4:5]" in ln for ln in lines)
    rng = np.random.default_rng(len(name) * 7)
    a_limbs = [(A >> (32 * i)) & M32 for i in range(4)]
    for s, inc in _states(rng):
        for m in (0, M32):
            u, v = int(rng.integers(0, 1 << 63)), int(rng.integers(0, 1 << 63))
            env = {"a0": a_limbs[0], "a1": a_limbs[1], "a2": a_limbs[2], "a3": a_limbs[3], "m": m,
                   "mm": m << 32 | m, "zs": 0, "u": u, "v": v, "vlo": v & M32, "vhi": v >> 32,
                   "s0": s & M32, "s1": (s >> 32) & M32, "s2": (s >> 64) & M32, "s3": s >> 96,
                   "c0": inc & M32, "c1": (inc >> 32) & M32, "c23": inc >> 64}
            lane = Lane(env, rng)
            for ln in lines:
                lane.run(ln)
            nxt = (s * A + inc) & M128
            raw = _raw(nxt)
            t = raw ^ (M64 if m else 0)
            e = lane.env
            assert e["s0"] | e["s1"] << 32 | e["s2"] << 64 | e["s3"] << 96 == nxt
            assert (e["zs"] != 0) == (raw == 0)
            assert e["u"] == (u + t) & M64
            if name == "pcg_draw_pair":
                assert e["vlo"] | e["vhi"] << 32 == (v - t) & M64
            elif name == "pcg_draw_pair_a":
                assert e["v"] == (v + t) & M64


def test_draw_instruction_budget():
    """The committed header's per-block VALU counts: 48-50 per
    two pair draws, 46 per two one-sided draws, no s_nop padding, and the
    header matches what the generator emits today."""
    import subprocess
    import sys

    text = open(os.path.join(ROOT, "sfl_amd", "csrc", "sa_draw2.h")).read()
    counts = dict(re.findall(r"// (pcg_draw2_\w+): (\d+) VALU \+ 0 s_nop", text))
    assert {k: int(v) for k, v in counts.items()} == {
        "pcg_draw2_pair_ss": 50, "pcg_draw2_pair_sa": 49, "pcg_draw2_pair_as": 49, "pcg_draw2_pair_aa": 48,
        "pcg_draw2_one": 46, "pcg_draw2_one_same": 46}
    gen = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_draw2.py")],
                         capture_output=True, text=True, check=True).stdout
    assert gen == text, "sa_draw2.h is stale: regenerate with tools/gen_draw2.py"
