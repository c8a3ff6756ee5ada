# Draw-loop microbenchmark of both draw forms (per-tile zero test in both),
# the W-rank rehearsal, then the whole GPU suite on the shift-rotation build.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_rots
rm -f gpurun_out/ab_rots/draw_issue2.txt
for exe in draw_issue_prev draw_issue draw_issue_prev draw_issue; do
  echo "== $exe" >> gpurun_out/ab_rots/draw_issue2.txt
  timeout -k 10 60 tools/microbench/$exe "dual pair28 E2" 2 >> gpurun_out/ab_rots/draw_issue2.txt 2>&1 || exit 1
  timeout -k 10 60 tools/microbench/$exe "dual one7 E2" 8 >> gpurun_out/ab_rots/draw_issue2.txt 2>&1 || exit 1
done
cat gpurun_out/ab_rots/draw_issue2.txt
timeout -k 10 900 python -u -m pytest -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/ab_rots/pytest2.log 2>&1
rc=$?
grep -E "passed|failed" gpurun_out/ab_rots/pytest2.log | tail -3
grep -A 30 "^____" gpurun_out/ab_rots/pytest2.log | head -80
exit $rc
