#!/usr/bin/env python3
"""Rough loop live-in VGPR census for one kernel in a hipcc .s file.
usage: loopregs.py file.s kernel_symbol"""
import re, sys
src, sym = sys.argv[1], sys.argv[2]
lines = open(src).read().split("\n")
s = next(i for i, l in enumerate(lines) if l.startswith(sym + ":"))
e = next(i for i in range(s, len(lines)) if "s_endpgm" in lines[i])
k = lines[s:e + 1]
labels = {l.split(":")[0]: i for i, l in enumerate(k) if re.match(r"^\.LBB\w+:", l)}
# loops: a branch to an earlier label
loops = []
for i, l in enumerate(k):
    m = re.search(r"s_(cbranch_\w+|branch)\s+(\.LBB\w+)", l)
    if m and m.group(2) in labels and labels[m.group(2)] < i:
        loops.append((labels[m.group(2)], i))
def regs(tok):
    out = []
    for m in re.finditer(r"v\[(\d+):(\d+)\]|\bv(\d+)\b", tok):
        out += [int(m.group(3))] if m.group(3) else list(range(int(m.group(1)), int(m.group(2)) + 1))
    return out
for (a, b) in loops:
    body = k[a:b + 1]
    written, livein = set(), set()
    nv = 0
    for l in body:
        l = l.split(";")[0].strip()
        if not l or l.endswith(":"):
            continue
        parts = l.split(None, 1)
        if len(parts) < 2:
            continue
        op, args = parts
        if op.startswith("v_"):
            nv += 1
        a_ = [x.strip() for x in re.split(r",(?![^\[]*\])", args)]
        if op.startswith(("global_store", "buffer_store", "ds_write", "flat_store", "global_atomic", "s_", "v_cmp", "v_cmpx")):
            dst, srcs = [], a_
        else:
            dst, srcs = regs(a_[0]), a_[1:]
        for t in srcs:
            for r in regs(t):
                if r not in written:
                    livein.add(r)
        written.update(dst)
    print(f"loop lines {a}-{b}: {b-a} lines, {nv} VALU, live-in VGPRs {len(livein)}")
