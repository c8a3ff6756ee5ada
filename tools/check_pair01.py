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

usage: python tools/check_pair01.py FILE.s [...]   (exit 1 on a violation)
"""
import re
import sys

MAD = re.compile(r"v_mad_u64_u32 v\[(\d+):(\d+)\], s\[\d+:\d+\], v(\d+), v\d+, s\[\d+:\d+\]")
ADD = re.compile(r"v_add_co_u32_e64 v(\d+), s\[\d+:\d+\], v(\d+), v\d+")


def check(path):
    text = open(path).read()
    bad, blocks, pairs = [], 0, 0
    for blk in re.findall(r";;#ASMSTART\n(.*?);;#ASMEND", text, re.S):
        if "v_mad_u64_u32" not in blk:
            continue
        blocks += 1
        adds = {int(a) for a, b in ADD.findall(blk) if a == b}
        for lo, hi, src in MAD.findall(blk):
            lo, hi, src = int(lo), int(hi), int(src)
            if lo < 20:  # draw scratch pairs (v0-v19, clobbered) hold column sums, not states
                continue
            pairs += 1
            if src != lo or hi not in adds:
                bad.append(f"pair v[{lo}:{hi}] limb-0 source v{src}, in-place limb-1 add {'yes' if hi in adds else 'NO'}")
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
