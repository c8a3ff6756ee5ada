#!/usr/bin/env python3
"""Build check of the draw's register aliasing (sa_draw2.h).

The draw keeps each state's limbs 0-1 in one 64-bit VGPR pair (asm operand
p01) and reads them through two 32-bit input operands s0 / s1 that the
compiler must place in that pair's two halves: the first column's mad
writes the pair in place and the limb-1 add completes its high half, so a
copy elsewhere would leave the state wrong.  This parses the device ISA of
every kernel (hipcc -S / --save-temps) and checks, for every draw block,
that each pair-writing mad reads its limb 0 from the pair's low register
and that the limb-1 add updates the pair's high register in place.

Run by the Makefile on every object that includes sa_draw2.h (the masking
kernels) and by __graft_entry__.build() on tools/microbench/draw_issue (the
draw-loop ceiling bench.py quotes).  The inline-asm contract cannot express
"this 32-bit input is the low half of that 64-bit operand", so a new hipcc
must pass this check before its build is used.

usage: python tools/check_pair01.py FILE.s [...]   (exit 1 on a violation)
"""
import re
import sys

MAD = re.compile(r"v_mad_u64_u32 v\[(\d+):(\d+)\], s\[\d+:\d+\], v(\d+), v\d+, s\[\d+:\d+\]")
ADD = re.compile(r"v_add_co_u32_e64 v(\d+), s\[\d+:\d+\], v(\d+), v\d+")
DEST = re.compile(r"^\s*v_\w+\s+v(?:\[(\d+):(\d+)\]|(\d+))")


def _dests(line):
    """VGPRs an instruction writes (its first operand)."""
    m = DEST.match(line)
    if not m:
        return set()
    if m.group(3) is not None:
        return {int(m.group(3))}
    return set(range(int(m.group(1)), int(m.group(2)) + 1))


def check(path):
    """For every pair-writing mad v[lo:hi] of a draw block: its limb-0 source
    is v{lo} (the pair's own low half), and the NEXT instruction in the block
    that writes v{hi} is the in-place limb-1 add on v{hi} itself -- so the
    high half the add completes is this pair's, not another draw's."""
    text = open(path).read()
    bad, blocks, pairs = [], 0, 0
    for blk in re.findall(r";;#ASMSTART\n(.*?);;#ASMEND", text, re.S):
        if "v_mad_u64_u32" not in blk:
            continue
        blocks += 1
        lines = [ln for ln in blk.splitlines() if ln.strip() and not ln.strip().startswith(";")]
        for i, ln in enumerate(lines):
            m = MAD.search(ln)
            if not m:
                continue
            lo, hi, src = (int(g) for g in m.groups())
            if lo < 20:  # draw scratch pairs (v0-v19, clobbered) hold column sums, not states
                continue
            pairs += 1
            nxt = next((lines[j] for j in range(i + 1, len(lines)) if hi in _dests(lines[j])), None)
            a = ADD.search(nxt) if nxt else None
            in_place = a is not None and int(a.group(1)) == hi and int(a.group(2)) == hi
            if src != lo or not in_place:
                bad.append(f"pair v[{lo}:{hi}] limb-0 source v{src}; next write of v{hi}: "
                           f"{nxt.strip() if nxt else 'none'}")
    return blocks, pairs, bad


def main():
    rc = 0
    for path in sys.argv[1:]:
        blocks, pairs, bad = check(path)
        print(f"{path}: {blocks} draw blocks, {pairs} state pairs written in place, {len(bad)} violations")
        for b in bad[:10]:
            print("  ", b)
        rc |= bool(bad) or (blocks > 0 and pairs == 0)
    sys.exit(rc)


if __name__ == "__main__":
    main()
