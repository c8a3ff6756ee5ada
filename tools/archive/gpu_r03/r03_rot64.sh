set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 100 tools/microbench/draw_ops > gpurun_out/draw_ops3.jsonl || exit 1
tail -6 gpurun_out/draw_ops3.jsonl
timeout -k 10 900 python -u -m pytest -x -q --timeout 300 --timeout-method thread tests/test_gpu_parity.py tests/test_gpu_fuzz.py tests/test_gpu_world_emulation.py > gpurun_out/t_rot64.log 2>&1 || { tail -40 gpurun_out/t_rot64.log; exit 1; }
tail -1 gpurun_out/t_rot64.log
bash tools/debug/ab_variants.sh ab_rot64 "base _alignbit" 8:1,8:2,8:4,8:8 4 > gpurun_out/ab_rot64.log 2>&1 || { tail gpurun_out/ab_rot64.log; exit 1; }
python tools/debug/ab_summary.py gpurun_out/ab_rot64/kb.jsonl 2>&1 | tail -12
