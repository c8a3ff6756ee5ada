#!/usr/bin/env python3
"""Register / spill census of the k_clients instantiations in a hipcc
-save-temps .s file.  usage: python tools/kregs.py sfl_amd/lib/obj/sa_clients_f32-hip-*.s"""
import re
import sys

for path in sys.argv[1:]:
    cur = {}
    for line in open(path):
        m = re.match(r"\s+\.name:\s+(\S+)", line)
        if m:
            cur = {"name": m.group(1)}
            continue
        m = re.match(r"\s+\.(sgpr_count|sgpr_spill_count|vgpr_count|vgpr_spill_count):\s+(\d+)", line)
        if m and cur:
            cur[m.group(1)] = int(m.group(2))
            if m.group(1) == "vgpr_spill_count":
                n = re.search(r"k_clientsI(\w+?)Li(\d+)ELi(\d+)E(?:Li(\d+)E)?", cur["name"])
                tag = f"{n.group(1)} L={n.group(2)} X={n.group(3)}" + (f" K={n.group(4)}" if n.group(4) not in (None, "0") else "") if n else cur["name"]
                print(f"{tag:22s} vgpr={cur.get('vgpr_count'):4d} vspill={cur['vgpr_spill_count']:3d} "
                      f"sgpr={cur.get('sgpr_count'):3d} sspill={cur.get('sgpr_spill_count')}")
