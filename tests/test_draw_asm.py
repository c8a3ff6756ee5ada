"""Host-side checks of the hand-scheduled PCG64 draw code (no GPU needed).

* sa_draw2.h is generated: re-running tools/gen_draw2.py reproduces the
  committed header byte for byte (no hand edits drift from the generator);
* every asm block in sa_clients_impl.h / sa_draw2.h honours the gfx950 rule
  the schedule relies on: an SGPR written by a VALU instruction (a carry-out
  or VCC) is read no earlier than the third instruction after the write;
* the draw's 128-bit step, restated from the asm's limb equations in
  Python integers, equals numpy's PCG64 transition and XSL-RR output.
"""
import os
import re
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
CSRC = os.path.join(ROOT, "sfl_amd", "csrc")


def test_draw2_header_matches_generator():
    out = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "gen_draw2.py")], capture_output=True,
                         text=True, check=True).stdout
    assert out == open(os.path.join(CSRC, "sa_draw2.h")).read()


def _asm_blocks():
    """Instruction lists of every asm string block (consecutive "..." lines)."""
    blocks = []
    for name in ("sa_clients_impl.h", "sa_draw2.h"):
        cur = []
        for line in open(os.path.join(CSRC, name)):
            m = re.search(r'"((?:v_|s_nop)[^"\\]*)(?:\\n\\t)?"', line)
            if m:
                cur.append(m.group(1).strip())
            elif cur and not line.strip().startswith(('"', "SA_PCG_DRAW_ASM")):
                blocks.append(cur)
                cur = []
        if cur:
            blocks.append(cur)
    return blocks


def _sgpr_operands(ins):
    ops = re.findall(r"%\[(\w+)\]|\b(vcc)\b", ins)
    return [a or b for a, b in ops]


CARRY = re.compile(r"^(k[123][ab]?|swb|vcc)$")


def test_valu_sgpr_write_read_distance():
    blocks = _asm_blocks()
    assert len(blocks) >= 4
    checked = 0
    for blk in blocks:
        last_write = {}
        for i, ins in enumerate(blk):
            if ins.startswith("s_nop"):
                continue
            op, _, args = ins.partition(" ")
            names = [x for x in _sgpr_operands(args) if CARRY.match(x)]
            if not names:
                continue
            # destinations: for VOP3b forms the carry-out is the 2nd operand,
            # VOPC e32 writes vcc; reads are the remaining carry operands
            parts = [p.strip() for p in re.split(r",(?![^\[]*\])", args)]
            writes, reads = set(), set()
            if op.startswith("v_cmp") and op.endswith("_e32"):
                writes.add("vcc")
            elif op.startswith("v_cmp"):
                writes.update(_sgpr_operands(parts[0]))
            elif op.startswith(("v_mad_u64_u32", "v_add_co", "v_addc_co", "v_sub_co", "v_subb_co")):
                writes.update(_sgpr_operands(parts[1]))
                for p in parts[2:]:
                    reads.update(x for x in _sgpr_operands(p) if CARRY.match(x))
            elif op.startswith("v_cndmask"):
                reads.update(x for x in _sgpr_operands(parts[-1]) if CARRY.match(x))
            for r in reads:
                if r in last_write:
                    assert i - last_write[r] >= 3, (blk[last_write[r]], ins)
                    checked += 1
            for w in writes:
                last_write[w] = i
    assert checked > 20


def test_limb_equations_equal_numpy_pcg64():
    """The asm computes S' = S*A + C from 32-bit limbs as E0 = s0a0 + c0,
    O1 = s0a1 + c1 + s1a0, E2 = s0a2 + s1a1 + s2a0 + C23 (mod 2^64),
    L3 = s0a3+s1a2+s2a1+s3a0 (mod 2^32); r = E0 + O1<<32 + E2<<64 + L3<<96
    mod 2^128, where E0 and the first O1 mad (s0a1 + c1) cannot carry out of
    64 bits.  Check against numpy."""
    M = (1 << 128) - 1
    A = 0x2360ED051FC65DA44385DF649FCCF645
    a = [(A >> (32 * i)) & 0xFFFFFFFF for i in range(4)]
    bg = np.random.PCG64(12345)
    st = bg.state["state"]
    s, inc = st["state"], st["inc"]
    gen = np.random.PCG64(12345)
    for _ in range(50):
        limbs = [(s >> (32 * i)) & 0xFFFFFFFF for i in range(4)]
        c0, c1, c23 = inc & 0xFFFFFFFF, (inc >> 32) & 0xFFFFFFFF, inc >> 64
        e0 = limbs[0] * a[0] + c0
        assert e0 < 1 << 64 and limbs[0] * a[1] + c1 < 1 << 64  # no carry-out
        o1 = limbs[0] * a[1] + c1 + limbs[1] * a[0]
        e2 = (limbs[0] * a[2] + limbs[1] * a[1] + limbs[2] * a[0] + c23) & ((1 << 64) - 1)
        l3 = (limbs[0] * a[3] + limbs[1] * a[2] + limbs[2] * a[1] + limbs[3] * a[0]) & 0xFFFFFFFF
        s = (e0 + (o1 << 32) + (e2 << 64) + (l3 << 96)) & M
        assert s == (s * 0 + ((limbs[0] | limbs[1] << 32 | limbs[2] << 64 | limbs[3] << 96) * A + inc) & M)
        hi, lo = s >> 64, s & ((1 << 64) - 1)
        x, r = hi ^ lo, hi >> 58
        out = ((x >> r) | (x << (64 - r))) & ((1 << 64) - 1)
        assert out == int(gen.random_raw())


def test_pair01_isa_check_flags_a_broken_alias(tmp_path):
    """tools/check_pair01.py (run by the Makefile on every build of the
    masking kernels) accepts a draw block whose state pair is written in
    place and rejects one where the compiler put limb 0 / limb 1 elsewhere."""
    good = """;;#ASMSTART
\tv_mad_u64_u32 v[2:3], s[40:41], v30, v41, s[4:5]
\tv_mad_u64_u32 v[30:31], s[42:43], v30, v40, s[6:7]
\tv_add_co_u32_e64 v31, s[44:45], v31, v2
;;#ASMEND
"""
    bad_src = good.replace("v[30:31], s[42:43], v30", "v[30:31], s[42:43], v28")
    bad_add = good.replace("v_add_co_u32_e64 v31, s[44:45], v31", "v_add_co_u32_e64 v29, s[44:45], v29")
    # the pair's high half overwritten between the mad and its in-place add:
    # an in-place add on v31 still exists, but it no longer completes this
    # mad's limb 1 (the order-aware check catches it)
    bad_order = good.replace("\tv_add_co_u32_e64 v31", "\tv_mov_b32 v31, v5\n\tv_add_co_u32_e64 v31")
    tool = os.path.join(ROOT, "tools", "check_pair01.py")
    rcs = []
    for i, text in enumerate((good, bad_src, bad_add, bad_order)):
        p = tmp_path / f"k{i}.s"
        p.write_text(text)
        rcs.append(subprocess.run([sys.executable, tool, str(p)], capture_output=True).returncode)
    assert rcs == [0, 1, 1, 1]
