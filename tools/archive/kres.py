#!/usr/bin/env python3
"""Summarise `hipcc -Rpass-analysis=kernel-resource-usage` remarks (stdin)."""
import re, sys
cur = None
rows = []
for line in sys.stdin:
    m = re.search(r"Function Name: (\S+)", line)
    if m:
        cur = {"name": m.group(1)}
        rows.append(cur)
        continue
    for key in ("VGPRs", "VGPRs Spill", "SGPRs Spill", "ScratchSize \\[bytes/lane\\]", "Occupancy \\[waves/SIMD\\]"):
        m = re.search(r"\s" + key + r": (\d+)", line)
        if m and cur is not None:
            cur[key.split()[0] + ("Spill" if "Spill" in key else "")] = int(m.group(1))
for r in rows:
    n = r["name"]
    m = re.search(r"k_clientsI(\w+?)Li(\d+)ELi(\d+)E(?:Li(\d+)E)?", n)
    tag = f"{m.group(1)} L={m.group(2)} X={m.group(3)}" + (f" K={m.group(4)}" if m.group(4) not in (None, "0") else "") if m else n
    print(f"{tag:28s} vgpr={r.get('VGPRs')} vspill={r.get('VGPRsSpill')} sspill={r.get('SGPRsSpill')} scratch={r.get('ScratchSize')} occ={r.get('Occupancy')}")
