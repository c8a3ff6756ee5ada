# A/B of the shift-rotation draw (product build) against the round-2
# alignbit draw (sfl_amd/lib/libsfl_sa_prev.so), then parity on the new build.
set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out/ab_rots
rm -f gpurun_out/ab_rots/draw_issue.txt
for exe in draw_issue_prev draw_issue draw_issue_prev draw_issue; do
  echo "== $exe" >> gpurun_out/ab_rots/draw_issue.txt
  timeout -k 10 60 tools/microbench/$exe "dual pair28 E2" 2 >> gpurun_out/ab_rots/draw_issue.txt 2>&1 || exit 1
  timeout -k 10 60 tools/microbench/$exe "dual one7 E2" 8 >> gpurun_out/ab_rots/draw_issue.txt 2>&1 || exit 1
done
cat gpurun_out/ab_rots/draw_issue.txt
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_rejection.py > gpurun_out/ab_rots/pytest_parity.log 2>&1 || { tail -40 gpurun_out/ab_rots/pytest_parity.log; exit 1; }
tail -1 gpurun_out/ab_rots/pytest_parity.log
bash tools/debug/ab_variants.sh ab_rots "_prev base" 8:1,8:2,8:4,8:8 4 > gpurun_out/ab_rots.log 2>&1 || { tail gpurun_out/ab_rots.log; exit 1; }
python tools/debug/ab_summary.py gpurun_out/ab_rots/kb.jsonl 2>&1 | tail -12
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests -m gpu > gpurun_out/ab_rots/pytest.log 2>&1 || { tail -40 gpurun_out/ab_rots/pytest.log; exit 1; }
tail -2 gpurun_out/ab_rots/pytest.log
