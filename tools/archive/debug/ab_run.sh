# A/B of the current library against sfl_amd/lib/libsfl_sa_prev.so (the
# previous commit's build), interleaved, then the GPU parity suite.
set -e
mkdir -p gpurun_out/ab
rm -f gpurun_out/ab/kb.jsonl
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/ab/pytest.log 2>&1
for v in _prev "" _prev ""; do
  SFL_SA_LIB=sfl_amd/lib/libsfl_sa${v}.so timeout -k 10 120 python -u tools/kernel_bench.py --rounds 5 >> gpurun_out/ab/kb.jsonl 2>/dev/null
done
timeout -k 10 100 tools/microbench/draw_issue > gpurun_out/ab/draw_issue.txt 2>&1
