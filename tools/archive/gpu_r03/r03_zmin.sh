# A/B of the raw == 0 test in the shift-rotation draw: SALU-OR-ed 64-bit
# compares (product build) vs the per-lane v_bitop3 + v_min3 minimum
# (libsfl_sa_zmin.so), with the round-2 alignbit draw (libsfl_sa_prev.so).
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_zmin
rm -f gpurun_out/ab_zmin/draw_issue.txt
for exe in draw_issue_prev draw_issue draw_issue_zmin draw_issue_prev draw_issue draw_issue_zmin; do
  echo "== $exe" >> gpurun_out/ab_zmin/draw_issue.txt
  timeout -k 10 60 tools/microbench/$exe "dual pair28 E2" 2 >> gpurun_out/ab_zmin/draw_issue.txt 2>&1 || exit 1
done
cat gpurun_out/ab_zmin/draw_issue.txt
bash tools/debug/ab_variants.sh ab_zmin "_prev base _zmin" 8:1,8:2,8:4,8:8 4 > gpurun_out/ab_zmin.log 2>&1 || { tail gpurun_out/ab_zmin.log; exit 1; }
python tools/debug/ab_summary.py gpurun_out/ab_zmin/kb.jsonl 2>&1 | tail -12
