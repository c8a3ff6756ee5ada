#!/usr/bin/env python3
"""Instruction mix of a kernel's hottest loop in a hipcc --save-temps .s file.

usage: python tools/isa_loop.py file.s KERNEL_SUBSTRING
Finds the longest backward branch in the kernel (the tile loop) and counts
VALU / SALU / LDS / VMEM / waitcnt instructions between target and branch."""
import collections
import re
import sys


def main():
    path, sub = sys.argv[1], sys.argv[2]
    src = open(path).read()
    names = [m for m in re.findall(r'^(_Z\S*):', src, re.M) if sub in m and not m.endswith('$local')]
    name = names[0]
    body = src[src.index(name + ':'):]
    body = body[:body.index('.Lfunc_end')]
    lines = [l.split(';')[0].strip() for l in body.split('\n')]
    labels = {l[:-1]: i for i, l in enumerate(lines) if re.match(r'^\.LBB\S+:$', l)}
    best = None
    for i, l in enumerate(lines):
        m = re.match(r's_(?:cbranch_\w+|branch)\s+(\.LBB\S+)', l)
        if m and labels.get(m.group(1), 1 << 30) < i:
            span = (labels[m.group(1)], i)
            if best is None or span[1] - span[0] > best[1] - best[0]:
                best = span
    lo, hi = best
    cnt = collections.Counter()
    ops = collections.Counter()
    for l in lines[lo:hi + 1]:
        if not l or l.startswith('.') or l.endswith(':'):
            continue
        op = l.split()[0]
        ops[op] += 1
        if op.startswith('v_'):
            cnt['valu'] += 1
        elif op.startswith('s_waitcnt'):
            cnt['waitcnt'] += 1
        elif op.startswith('s_'):
            cnt['salu'] += 1
        elif op.startswith('ds_'):
            cnt['lds'] += 1
        elif op.startswith(('buffer_', 'global_')):
            cnt['vmem'] += 1
        else:
            cnt['other'] += 1
    print(name, 'loop lines', lo, hi)
    print(dict(cnt))
    for op, c in ops.most_common(40):
        print(f'{c:6d} {op}')


if __name__ == '__main__':
    main()
