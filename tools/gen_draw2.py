#!/usr/bin/env python3
"""Generates sfl_amd/csrc/sa_draw2.h: two PCG64 draws (two independent mask
streams, same multiplier) as ONE hand-scheduled inline-asm block, their
instruction streams interleaved so every dependent pair of one stream sits at
least two issue slots apart (the other stream's instruction fills the gap).

The single-draw schedule is SA_PCG_DRAW_ASM in sa_clients_impl.h; this script
keeps its instructions except one -- limbs 0-1 of a state are one VGPR pair
that the first column's mad (moved after the last read of limbs 0-1)
writes in place, so the single draw's v_mov of the new limb 0 is gone --
renames stream B onto its own scratch VGPRs
(v10-v19), carry SGPR pairs and a swap mask in an SGPR pair instead of VCC,
merges the two raw==0 running minimums into one v_min3, and checks the gfx950
rule the single draw already follows: a VALU-written SGPR (carry, VCC) is
read no earlier than the third instruction after the write (s_nop padding is
inserted where the interleave alone does not give that).

Accumulation: the client accumulators are 64-bit VGPR pairs.  The draw is
added with ONE v_lshl_add_u64 (measured at the issue cost of one v_add_co,
tools/microbench/op_rate.hip: the v_add_co + v_addc pair costs two); the
second client of an internal pair either also adds (kernel stores it
negated) or subtracts with v_sub_co + v_subb on the pair's 32-bit halves.
Functions are emitted per (stream a, stream b) second-client mode: "s"
subtract, "a" add.

First touch: each function is a template over F, a bit set of the block's
accumulators (bit 0 ua, 1 va, 2 ub, 3 vb) that the tile has not touched yet.
A first-touched accumulator is not read: its add takes the client's bias
constant from an SGPR pair instead (v_lshl_add_u64 u, t, 0, s[bias]), so the
kernel needs no per-tile v_mov to preset the accumulators.  Subtracting
partners (v_sub_co + v_subb on halves) have no first-touch form: the subb
would read two SGPRs (bias and borrow), one more than the gfx9 constant bus
allows; the kernel's schedule orders groups so that no client is first
touched as a subtracting partner (and presets any that would be).

The s0 / s1 operands are declared as inputs although the pair-writing mad
overwrites their registers: the inline-asm contract has no way to say "the
low half of that 64-bit operand", so correctness rests on the register
allocator placing them in the pair's halves.  tools/check_pair01.py verifies
that on the ISA of every build (the library's masking kernels and
tools/microbench/draw_issue); a hipcc upgrade must pass it before its build
is used, and a failing build leaves no object behind.

usage: python tools/gen_draw2.py > sfl_amd/csrc/sa_draw2.h
"""

import re
import sys

# Limbs 0-1 of each state live in one 64-bit VGPR pair (operand p01, "+v");
# the first column's mad writes that pair directly (its low word IS the new
# limb 0, its high word the partial limb 1 that the add then completes in
# place), so the draw needs no v_mov.  The 32-bit operands s0 / s1 are
# inputs the compiler places in the pair's two halves (reads of limbs 0-1
# all come before the pair is written) -- build-checked by
# tools/check_pair01.py on the ISA.  --no-pair01 emits the earlier form
# (limbs in four 32-bit operands, the new limb 0 moved in from scratch).
PAIR01 = "--no-pair01" not in sys.argv
# --rot64: XSL-RR's 64-bit rotation by r = s3 >> 26 as two 64-bit shifts and
# an OR (x >> r | x << (64 - r) & 63, exact for r = 0 too: x | x) instead of
# two v_alignbit (rotating by r & 31) + a v_cmp on bit 31 of s3 + two
# v_cndmask swapping the halves when r >= 32.  The same instruction count,
# 5.6 fewer cycles per draw by the per-form issue costs
# (tools/microbench/draw_ops.hip), but measured neutral in the kernel
# (profiles/r03/ab_rot64_kb.jsonl: every per-rank shape within +-1.5 %), so
# the default stays the alignbit form.  Both are pinned to numpy on the CPU
# by tests/test_draw_emulation.py.
ROT64 = "--rot64" in sys.argv
# Default form (ROTS): XSL-RR's rotation as two 64-bit shifts whose parts are
# ADDED by one v_lshl_add_u64 -- y = x >> r, z = x << (63 - r), t = (z << 1)
# + y: the two parts have disjoint bits, so + is |, and for r = 0 the shift
# by one more bit makes z's part vanish (t = x) -- 5 instructions (shift
# amount, its complement, two shifts, the join) instead of the alignbit
# form's 6 (shift amount, two v_alignbit, v_cmp, two v_cndmask); and the
# raw == 0 test as ONE 64-bit compare of x with the sign mask pair (x == m:m
# <=> raw == 0) into VCC / an SGPR pair, OR-ed into a wave-wide hit mask on
# the SALU (which issues beside the other wave's VALU), instead of a v_bitop3
# "all equal" per draw + a v_min3 per two draws: 1.5 VALU per draw fewer in
# all.  --alignbit emits the round-2 form.
ROTS = not ROT64 and "--alignbit" not in sys.argv
# --zmin (with ROTS): the shift rotation, but the round-2 raw == 0 test (a
# v_bitop3 "all equal" per draw + one v_min3 per two draws into a per-lane
# running minimum) instead of the SALU-OR-ed 64-bit compares -- one VALU more
# per two draws, no SALU: for A/B (tools/microbench/draw_ops: a compare +
# s_or_b64 pair issues at 7.5 cycles, the compare alone at 4.5).
ZMIN_FORM = ROTS and "--zmin" in sys.argv

# one draw: (asm, sgpr_writes, sgpr_reads); {..} fields are renamed per stream
DRAW = [
    ("v_mad_u64_u32 v[{v0}:{v1}], %[{k1}], %[{s0}], %[a0], %[{c0}]", {"k1"}, set()),
    ("v_mad_u64_u32 v[{v2}:{v3}], %[{k3}], %[{s0}], %[a1], %[{c1}]", {"k3"}, set()),
    ("v_mad_u64_u32 v[{v4}:{v5}], %[{k3}], %[{s0}], %[a2], %[{c23}]", {"k3"}, set()),
    ("v_mul_lo_u32 v{v6}, %[{s0}], %[a3]", set(), set()),
    ("v_mad_u64_u32 v[{v2}:{v3}], %[{k2}], %[{s1}], %[a0], v[{v2}:{v3}]", {"k2"}, set()),
    ("v_mad_u64_u32 v[{v4}:{v5}], %[{k3}], %[{s1}], %[a1], v[{v4}:{v5}]", {"k3"}, set()),
    ("v_mad_u64_u32 v[{v6}:{v7}], %[{k3}], %[{s1}], %[a2], v[{v6}:{v7}]", {"k3"}, set()),
    ("v_mad_u64_u32 v[{v4}:{v5}], %[{k3}], %[{s2}], %[a0], v[{v4}:{v5}]", {"k3"}, set()),
    ("v_mad_u64_u32 v[{v6}:{v7}], %[{k3}], %[{s2}], %[a1], v[{v6}:{v7}]", {"k3"}, set()),
    ("v_mad_u64_u32 v[{v6}:{v7}], %[{k3}], %[{s3}], %[a0], v[{v6}:{v7}]", {"k3"}, set()),
    ("v_add_co_u32_e64 %[{s1}], %[{k3}], v{v1}, v{v2}", {"k3"}, set()),
    ("v_addc_co_u32_e64 %[{s3}], %[{k2}], v{v5}, v{v6}, %[{k2}]", {"k2"}, {"k2"}),
    ("v_mov_b32_e32 %[{s0}], v{v0}", set(), set()),
    ("v_addc_co_u32_e64 %[{s2}], %[{k2}], v{v4}, v{v3}, %[{k3}]", {"k2"}, {"k3"}),
    ("v_bitop3_b32 v{v0}, %[{s0}], %[{s2}], %[{m}] bitop3:0x96", set(), set()),
    ("v_addc_co_u32_e64 %[{s3}], %[{k3}], %[{s3}], 0, %[{k2}]", {"k3"}, {"k2"}),
    ("v_bitop3_b32 v{v1}, %[{s1}], %[{s3}], %[{m}] bitop3:0x96", set(), set()),
    ("{cmp}", {"sw"}, set()),
    ("v_lshrrev_b32_e32 v{v2}, 26, %[{s3}]", set(), set()),
    ("v_bitop3_b32 v{v3}, v{v0}, v{v1}, %[{m}] bitop3:0x7e", set(), set()),
    ("v_alignbit_b32 v{v4}, v{v1}, v{v0}, v{v2}", set(), set()),
    ("v_alignbit_b32 v{v5}, v{v0}, v{v1}, v{v2}", set(), set()),
    ("ZMIN", set(), set()),
    ("{cnd_lo}", set(), {"sw"}),
    ("VSUBLO", {"k2"}, set()),
    ("{cnd_hi}", set(), {"sw"}),
    ("v_lshl_add_u64 %[{u}], v[{v6}:{v7}], 0, %[{u}]", set(), set()),
    ("VADD", set(), set()),
    ("VSUBHI", {"k2"}, {"k2"}),
]


ROT64_STEPS = [  # replaces {cmp} .. {cnd_hi} of DRAW (the rotation), zero test and accumulate kept in place
    ("v_lshrrev_b32_e32 v{v2}, 26, %[{s3}]", set(), set()),
    ("v_bitop3_b32 v{v3}, v{v0}, v{v1}, %[{m}] bitop3:0x7e", set(), set()),
    ("v_sub_u32_e32 v{v8}, 64, v{v2}", set(), set()),
    ("v_lshrrev_b64 v[{v4}:{v5}], v{v2}, v[{v0}:{v1}]", set(), set()),
    ("ZMIN", set(), set()),
    ("v_lshlrev_b64 v[{v6}:{v7}], v{v8}, v[{v0}:{v1}]", set(), set()),
    ("v_or_b32_e32 v{v6}, v{v6}, v{v4}", set(), set()),
    ("VSUBLO", {"k2"}, set()),
    ("v_or_b32_e32 v{v7}, v{v7}, v{v5}", set(), set()),
]


ROTS_STEPS = [  # replaces {cmp} .. {cnd_hi} and the zero test of DRAW; accumulate kept in place
    ("v_lshrrev_b32_e32 v{v2}, 26, %[{s3}]", set(), set()),
    ("v_xor_b32_e32 v{v3}, 63, v{v2}", set(), set()),
    ("{zcmp}", {"z"}, set()),
    ("v_lshrrev_b64 v[{v4}:{v5}], v{v2}, v[{v0}:{v1}]", set(), set()),
    ("v_lshlrev_b64 v[{v6}:{v7}], v{v3}, v[{v0}:{v1}]", set(), set()),
    ("{zor}", set(), {"z"}),
    ("v_lshl_add_u64 v[{v6}:{v7}], v[{v6}:{v7}], 1, v[{v4}:{v5}]", set(), set()),
    ("VSUBLO", {"k2"}, set()),
]


ROTS_ZMIN_STEPS = [  # ROTS_STEPS with the per-lane minimum zero test
    ("v_lshrrev_b32_e32 v{v2}, 26, %[{s3}]", set(), set()),
    ("v_bitop3_b32 v{v8}, v{v0}, v{v1}, %[{m}] bitop3:0x7e", set(), set()),
    ("v_xor_b32_e32 v{v3}, 63, v{v2}", set(), set()),
    ("v_lshrrev_b64 v[{v4}:{v5}], v{v2}, v[{v0}:{v1}]", set(), set()),
    ("ZMIN", set(), set()),
    ("v_lshlrev_b64 v[{v6}:{v7}], v{v3}, v[{v0}:{v1}]", set(), set()),
    ("v_lshl_add_u64 v[{v6}:{v7}], v[{v6}:{v7}], 1, v[{v4}:{v5}]", set(), set()),
    ("VSUBLO", {"k2"}, set()),
]


def draw_steps():
    """DRAW with the rotation (and zero test) in the form the flags select."""
    if ROTS:
        i0 = DRAW.index(("{cmp}", {"sw"}, set()))
        i1 = DRAW.index(("{cnd_hi}", set(), {"sw"}))
        return DRAW[:i0] + (ROTS_ZMIN_STEPS if ZMIN_FORM else ROTS_STEPS) + DRAW[i1 + 1:]
    if not ROT64:
        return DRAW
    i0 = DRAW.index(("{cmp}", {"sw"}, set()))
    i1 = DRAW.index(("{cnd_hi}", set(), {"sw"}))
    return DRAW[:i0] + ROT64_STEPS + DRAW[i1 + 1:]


def stream(tag, base, vmode, acc_u, acc_v):
    """vmode: None (no second client), "s" (subtract) or "a" (add)."""
    f = {"s0": f"s0{tag}", "s1": f"s1{tag}", "s2": f"s2{tag}", "s3": f"s3{tag}",
         "k1": f"k1{tag}", "k2": f"k2{tag}", "k3": f"k3{tag}",
         "c0": f"c0{tag}", "c1": f"c1{tag}", "c23": f"c23{tag}", "m": f"m{tag}", "u": acc_u}
    for i in range(10):
        f[f"v{i}"] = str(base + i)
    if tag == "a":
        f["zcmp"] = f"v_cmp_eq_u64_e32 vcc, %[mma], v[{base}:{base + 1}]"
        f["zor"] = "s_or_b64 %[zh], %[zh], vcc"
    else:
        f["zcmp"] = f"v_cmp_eq_u64_e64 %[swb], %[mmb], v[{base}:{base + 1}]"
        f["zor"] = "s_or_b64 %[zh], %[zh], %[swb]"
    if tag == "a":
        f["cmp"] = f"v_cmp_gt_i32_e32 vcc, 0, %[s3a]"
        f["cnd_lo"] = f"v_cndmask_b32_e32 v{base + 6}, v{base + 4}, v{base + 5}, vcc"
        f["cnd_hi"] = f"v_cndmask_b32_e32 v{base + 7}, v{base + 5}, v{base + 4}, vcc"
    else:
        f["cmp"] = f"v_cmp_gt_i32_e64 %[swb], 0, %[s3b]"
        f["cnd_lo"] = f"v_cndmask_b32_e64 v{base + 6}, v{base + 4}, v{base + 5}, %[swb]"
        f["cnd_hi"] = f"v_cndmask_b32_e64 v{base + 7}, v{base + 5}, v{base + 4}, %[swb]"
    out = []
    draw = draw_steps()
    if PAIR01:
        f["p01"] = f"p01{tag}"
        e0 = None
        draw = []
        for asm, w, r in draw_steps():
            if asm.startswith("v_mad_u64_u32 v[{v0}:{v1}]"):
                e0 = (asm.replace("v[{v0}:{v1}]", "%[{p01}]"), w, r)
                continue
            if asm.startswith("v_mov_b32_e32 %[{s0}]"):
                continue
            asm = asm.replace("v_add_co_u32_e64 %[{s1}], %[{k3}], v{v1}, v{v2}",
                              "v_add_co_u32_e64 %[{s1}], %[{k3}], %[{s1}], v{v2}")
            draw.append((asm, w, r))
            if asm.startswith("v_mad_u64_u32 v[{v6}:{v7}], %[{k3}], %[{s1}], %[a2]"):
                draw.append(e0)  # after the last read of limbs 0 and 1
    for asm, w, r in draw:
        if asm == "VADD":
            if vmode != "a":
                continue
            asm = f"v_lshl_add_u64 %[{acc_v}], v[{base + 6}:{base + 7}], 0, %[{acc_v}]"
        elif asm == "VSUBLO":
            if vmode != "s":
                continue
            asm = f"v_sub_co_u32_e64 %[{acc_v}lo], %[k2{tag}], %[{acc_v}lo], v{base + 6}"
        elif asm == "VSUBHI":
            if vmode != "s":
                continue
            asm = f"v_subb_co_u32_e64 %[{acc_v}hi], %[k2{tag}], %[{acc_v}hi], v{base + 7}, %[k2{tag}]"
        elif asm == "ZMIN":
            asm = "ZMIN"
        else:
            asm = asm.format(**f)
        out.append((asm, {f"{x}{tag}" for x in w}, {f"{x}{tag}" for x in r}))
    return out


def interleave(a, b):
    seq = []
    for i in range(max(len(a), len(b))):
        if i < len(a):
            seq.append(a[i])
        if i < len(b):
            seq.append(b[i])
    # the two raw==0 minimums become one v_min3 at B's ZMIN slot
    zs = [i for i, s in enumerate(seq) if s[0] == "ZMIN"]
    if zs:
        z = (8, 18) if ZMIN_FORM else (3, 13)
        seq[zs[1]] = (f"v_min3_u32 %[zmin], %[zmin], v{z[0]}, v{z[1]}", set(), set())
        del seq[zs[0]]
    # hazard check: reader index - last writer index >= 3, else pad with s_nop
    out = []
    last_w = {}
    for asm, w, r in seq:
        need = max([last_w[x] + 3 for x in r if x in last_w] or [0])
        while len(out) < need:
            out.append(("s_nop 0", set(), set()))
            need = max([last_w[x] + 3 for x in r if x in last_w] or [0])
        for x in w:
            last_w[x] = len(out)
        out.append((asm, w, r))
    return out


def valid_flags(vma, vmb, same_acc):
    """First-touch bit sets F a function supports (see the docstring)."""
    out = []
    for f in range(16):
        if (f & 2) and vma != "a":
            continue
        if (f & 8) and vmb != "a":
            continue
        if same_acc and (f & 4):
            continue
        out.append(f)
    return out


def block(vma, vmb, same_acc, f):
    """(asm lines, outputs, inputs) of one variant."""
    acc_ua, acc_va = "ua", "va"
    acc_ub, acc_vb = ("ua", None) if same_acc else ("ub", "vb")
    a = stream("a", 0, vma, acc_ua, acc_va)
    b = stream("b", 10, vmb, acc_ub, acc_vb)
    seq = interleave(a, b)
    first = {"ua": bool(f & 1), "va": bool(f & 2), "ub": bool(f & 4), "vb": bool(f & 8)}
    lines = []
    for asm, _, _ in seq:
        m = re.match(r"v_lshl_add_u64 %\[(\w+)\], (v\[\d+:\d+\]), 0, %\[(\w+)\]$", asm)
        if m and m.group(1) == m.group(3) and first.get(m.group(1)):
            if same_acc and m.group(1) == "ua" and any("%[bua]" in x for x in lines):
                pass  # second cross stream of the same client: adds to the first's result
            else:
                asm = f"v_lshl_add_u64 %[{m.group(1)}], {m.group(2)}, 0, %[b{m.group(1)}]"
        lines.append(asm)
    u64 = ["ua"] + ([] if same_acc else ["ub"]) + [x for x, m in (("va", vma), ("vb", vmb)) if m == "a"]
    split = [x for x, m in (("va", vma), ("vb", vmb)) if m == "s"]
    accs = ["ua"] + (["va"] if vma else []) + ([] if same_acc else ["ub"] + (["vb"] if vmb else []))
    zout = '[zh] "+s"(zh)' if ROTS and not ZMIN_FORM else '[zmin] "+v"(zh)'
    outs = ['[s0a] "+v"(s0a)', '[s1a] "+v"(s1a)', '[s2a] "+v"(s2a)', '[s3a] "+v"(s3a)',
            '[s0b] "+v"(s0b)', '[s1b] "+v"(s1b)', '[s2b] "+v"(s2b)', '[s3b] "+v"(s3b)', zout]
    if PAIR01:
        outs = ['[p01a] "+v"(p01a)', '[s2a] "+v"(s2a)', '[s3a] "+v"(s3a)',
                '[p01b] "+v"(p01b)', '[s2b] "+v"(s2b)', '[s3b] "+v"(s3b)', zout]
    outs += [f'[{x}] "=&v"({x})' if first[x] else f'[{x}] "+v"({x})' for x in accs if x in u64]
    outs += [f'[{x}{h}] "+v"({x}{h})' for x in split for h in ("lo", "hi")]
    outs += [f'[{k}] "=&s"({k})' for k in ("k1a", "k2a", "k3a", "k1b", "k2b", "k3b", "swb")]
    ins = ['[a0] "v"(a0)', '[a1] "v"(a1)', '[a2] "v"(a2)', '[a3] "v"(a3)',
           '[c0a] "s"(ia.w0)', '[c1a] "s"(ia.w1)', '[c23a] "s"(ia.hi)', '[ma] "s"(ma)',
           '[c0b] "s"(ib.w0)', '[c1b] "s"(ib.w1)', '[c23b] "s"(ib.hi)', '[mb] "s"(mb)']
    if ROTS and not ZMIN_FORM:
        ins += ['[mma] "s"(mma)', '[mmb] "s"(mmb)']
    ins += [f'[b{x}] "s"(b{x})' for x in accs if x in u64 and first[x]]
    if PAIR01:
        ins += ['[s0a] "v"(s0a)', '[s1a] "v"(s1a)', '[s0b] "v"(s0b)', '[s1b] "v"(s1b)']
    return lines, outs, ins, seq, split, accs


def emit(name, vma, vmb, same_acc):
    flags = valid_flags(vma, vmb, same_acc)
    _, _, _, seq, split, accs = block(vma, vmb, same_acc, 0)
    n_valu = sum(1 for s in seq if s[0].startswith("v_"))
    n_nop = sum(1 for s in seq if s[0].startswith("s_nop"))
    lines = []
    lines.append(f"// {name}: {n_valu} VALU + {n_nop} s_nop for two draws; first-touch sets F in {{{', '.join(map(str, flags))}}}")
    st_params = (["uint64_t& p01a", "uint32_t& s2a", "uint32_t& s3a", "uint64_t& p01b", "uint32_t& s2b", "uint32_t& s3b"]
                 if PAIR01 else
                 ["uint32_t& s0a", "uint32_t& s1a", "uint32_t& s2a", "uint32_t& s3a",
                  "uint32_t& s0b", "uint32_t& s1b", "uint32_t& s2b", "uint32_t& s3b"])
    params = st_params + [
              "uint32_t a0", "uint32_t a1", "uint32_t a2", "uint32_t a3",
              "const Inc& ia", "uint32_t ma", "const Inc& ib", "uint32_t mb",
              "ZeroAcc& zh"] + [f"uint64_t& {x}" for x in accs] + [f"uint64_t b{x}" for x in accs]
    lines.append("template <int F>")
    lines.append(f"__device__ __forceinline__ void {name}(" + ", ".join(params) + ") {")
    lines.append("  uint64_t k1a, k2a, k3a, k1b, k2b, k3b, swb;")
    if ROTS and not ZMIN_FORM:
        lines.append("  // the sign masks as SGPR pairs (m:m) for the 64-bit raw == 0 compare")
        lines.append("  const uint64_t mma = (uint64_t)ma << 32 | ma, mmb = (uint64_t)mb << 32 | mb;")
    for x in split:
        lines.append(f"  uint32_t {x}lo = (uint32_t){x}, {x}hi = (uint32_t)({x} >> 32);")
    for x in accs:
        lines.append(f"  (void)b{x};")
    if PAIR01:
        lines.append("  // limbs 0 / 1 as 32-bit inputs: the halves of p01 (aliasing build-checked)")
        for t in "ab":
            lines.append(f"  const uint32_t s0{t} = (uint32_t)p01{t}, s1{t} = (uint32_t)(p01{t} >> 32);")
    for i, f in enumerate(flags):
        body, outs, ins, _, _, _ = block(vma, vmb, same_acc, f)
        lines.append(f"  {'if' if i == 0 else '} else if'} constexpr (F == {f}) {{")
        lines.append("    asm volatile(")
        for asm in body:
            lines.append(f'        "{asm}\\n\\t"')
        lines.append("        : " + ", ".join(outs))
        lines.append("        : " + ", ".join(ins))
        # ROTS: the SALU OR of the zero test writes SCC
        clob = ['"vcc"'] + (['"scc"'] if ROTS and not ZMIN_FORM else []) + [f'"v{i}"' for i in range(20)]
        lines.append("        : " + ", ".join(clob) + ");")
    lines.append("  } else {")
    lines.append("    __builtin_trap();  // no such first-touch variant (the kernel's schedule never asks)")
    lines.append("  }")
    for x in split:
        lines.append(f"  {x} = ((uint64_t){x}hi << 32) | {x}lo;")
    lines.append("}")
    return "\n".join(lines)


def main():
    print("// sa_draw2.h -- GENERATED by tools/gen_draw2.py; do not edit.")
    print("// Two interleaved PCG64 draws per asm block (see the generator's docstring);")
    print("// operand conventions as pcg_draw_pair / pcg_draw_one in sa_clients_impl.h.")
    print("#pragma once")
    print("#include <stdint.h>")
    print()
    print("namespace sa {")
    print()
    print("// A stream's increment as the draw's three SGPR addends: the two low words")
    print("// zero-extended (so s0*a0 + w0 and s0*a1 + w1 cannot carry) and the high half.")
    print("struct Inc {")
    print("  uint64_t w0, w1, hi;")
    print("};")
    print()
    form = ("rots_zmin" if ZMIN_FORM else "rots") if ROTS else ("rot64" if ROT64 else "alignbit")
    print(f'#define SA_DRAW2_FORM "{form}"')
    print()
    print("// The paired draws' running raw == 0 test (numpy re-draws a raw 0), kept per")
    print("// tile by the caller: zero_acc_init() before the tile's draws, zero_acc_hit()")
    print("// after them.")
    if ROTS and not ZMIN_FORM:
        print("// Here: the 64-bit compares OR-ed on the SALU into a wave-wide SGPR mask")
        print("// (bit l: a draw of lane l was 0); zero_acc_hit is wave-uniform.  (Kept per")
        print("// tile: a kernel-long SGPR accumulator fails to compile -- illegal VGPR to")
        print("// SGPR copy -- in the kernels with VGPR digests.)")
        print("typedef uint64_t ZeroAcc;")
        print("__device__ __forceinline__ ZeroAcc zero_acc_init() { return 0; }")
        print("__device__ __forceinline__ bool zero_acc_hit(ZeroAcc z) { return z != 0; }")
    else:
        print("// Here: a per-lane running minimum, 0 iff a draw of this lane was 0.")
        print("typedef uint32_t ZeroAcc;")
        print("__device__ __forceinline__ ZeroAcc zero_acc_init() { return 0xFFFFFFFFu; }")
        print("__device__ __forceinline__ bool zero_acc_hit(ZeroAcc z) { return z == 0; }")
    print()
    for ma in "sa":
        for mb in "sa":
            print(emit(f"pcg_draw2_pair_{ma}{mb}", ma, mb, same_acc=False))
            print()
    print(emit("pcg_draw2_one", None, None, same_acc=False))
    print()
    print(emit("pcg_draw2_one_same", None, None, same_acc=True))
    print()
    print("}  // namespace sa")


if __name__ == "__main__":
    main()
