#!/bin/bash
# SQ issue/stall census of the masking kernels (one rocprofv3 --pmc pass, 8 SQ
# counters + GRBM_GUI_ACTIVE) on the kernel_bench shapes.  Output CSV under
# gpurun_out/pmc_sq/.  usage: tools/pmc_sq.sh [shapes]   (default 8:1,8:8)
set -e
export TMPDIR=/tmp
SHAPES=${1:-8:1,8:8}
mkdir -p gpurun_out
timeout -s KILL 120 rocprofv3 --pmc SQ_WAVE_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY \
  SQ_ACTIVE_INST_VALU SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM GRBM_GUI_ACTIVE \
  --output-format csv -d gpurun_out/pmc_sq -o run -- \
  python3 tools/kernel_bench.py --shapes "$SHAPES" --rounds 1 --reps 2 > gpurun_out/pmc_sq.log 2>&1
python3 - <<'PY'
import csv, glob, collections
rows = []
for f in glob.glob("gpurun_out/pmc_sq/**/*counter_collection.csv", recursive=True):
    rows += list(csv.DictReader(open(f)))
by = collections.defaultdict(lambda: collections.defaultdict(list))
for r in rows:
    if "k_clients" not in r["Kernel_Name"]:
        continue
    by[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, d in by.items():
    m = {c: sum(v) / len(v) for c, v in d.items()}
    print(k[:60], {c: f"{v:.4g}" for c, v in sorted(m.items())})
    wc = m["SQ_WAVE_CYCLES"]
    print("   wait_any %.3f  wait_inst %.3f  active %.3f  active_valu %.3f  valu/instr-per-wave-cycle"
          % (m["SQ_WAIT_ANY"] / wc, m["SQ_WAIT_INST_ANY"] / wc, m["SQ_ACTIVE_INST_ANY"] / wc,
             m["SQ_ACTIVE_INST_VALU"] / wc))
PY
