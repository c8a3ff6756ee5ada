#!/bin/bash
# Round profile of the headline path (run on the GPU box from the repo root):
#   1. bench.py (default workload, then --extra) -> gpurun_out/bench*.jsonl
#   2. rocprofv3 --kernel-trace --stats of the same bench command
#   3. PMC passes, one counter group per run: FETCH_SIZE, WRITE_SIZE on
#      tools/kernel_bench.py over every per-rank shape (8 clients over 1, 2, 4, 8
#      GPUs at 100M element positions) + the k_sum_u64 calibration launch whose
#      bytes are known; the SQ issue census (tools/pmc_sq.sh)
# Copy what should be judged into profiles/<round>/ afterwards
# (tools/save_profiles.sh <round>).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench.jsonl 2> gpurun_out/bench.err
tail -1 gpurun_out/bench.jsonl
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- \
  python3 bench.py --cpu-baseline-seconds 0 > gpurun_out/bench_prof.jsonl 2> gpurun_out/bench_prof.err
tail -1 gpurun_out/bench_prof.jsonl
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- \
  python3 tools/kernel_bench.py --shapes 8:1,8:2,8:4,8:8 --rounds 1 --reps 2 --calib 8 --bipartite > gpurun_out/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- \
  python3 tools/kernel_bench.py --shapes 8:1,8:2,8:4,8:8 --rounds 1 --reps 2 --calib 8 --bipartite > gpurun_out/pmc_write.log 2>&1
tools/pmc_sq.sh 8:1,8:8 > /dev/null
timeout -k 10 120 python -u tools/kernel_bench.py --rounds 5 > gpurun_out/kb_shapes.jsonl
timeout -k 10 400 python bench.py --extra --cpu-baseline-seconds 0 > gpurun_out/bench_extra.jsonl 2> gpurun_out/bench_extra.err
echo PROFILE_OK
