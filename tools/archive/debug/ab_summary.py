#!/usr/bin/env python3
"""Summarise gpurun_out/<dir>/kb.jsonl from ab_variants.sh: median ms per (lib, shape)."""
import collections, json, sys
d = collections.defaultdict(list)
for line in open(sys.argv[1]):
    if not line.startswith("{"):
        continue
    r = json.loads(line)
    for c in r["cases"]:
        d[(r["lib"], c["C"], c["W"])].append(c["ms_median"])
for k in sorted(d):
    v = sorted(d[k])
    print(f"{k[0]:40s} C={k[1]} W={k[2]}  median {v[len(v)//2]:.4f} ms  all {' '.join(f'{x:.4f}' for x in v)}")
