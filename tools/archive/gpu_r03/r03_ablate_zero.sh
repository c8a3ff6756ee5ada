# Timing-only ablation of the paired draws' raw == 0 test (results of the
# variants are wrong for a raw 0 draw; never shipped): product build vs the
# same without the SALU ORs (_nozor) and without compare + ORs (_nocmp).
set -o pipefail
export TMPDIR=/tmp
bash tools/debug/ab_variants.sh ab_zero "base _nozor _nocmp" 8:1,8:8 3 > gpurun_out/ab_zero.log 2>&1 || { tail gpurun_out/ab_zero.log; exit 1; }
python tools/debug/ab_summary.py gpurun_out/ab_zero/kb.jsonl 2>&1 | tail -12
