#!/bin/bash
# Round profile of the headline path (run on the GPU box from the repo root):
#   1. bench.py (default workload, then --extra; and the --dist world-1
#      rehearsal timing every exchange design) -> gpurun_out/bench*.jsonl
#   2. rocprofv3 --kernel-trace --stats of the same bench command, and of the
#      server kernels (tools/server_bench.py)
#   3. PMC passes, one counter group per run: FETCH_SIZE, WRITE_SIZE on
#      tools/kernel_bench.py over every per-rank shape (8 clients over 1, 2, 4, 8
#      GPUs at 100M element positions) + the bipartite launch + the k_sum_u64
#      calibration launch whose bytes are known, and on tools/server_bench.py
#      (k_sum_u64, k_decode, k_sum_f64) and tools/dp_bench.py (the DP
#      pre-step kernels); the SQ issue census (tools/pmc_sq.sh)
#   4. microbenchmarks: per-instruction issue cost of the draw (draw_ops),
#      HBM streaming shapes (stream_rate)
# Copy what should be judged into profiles/<round>/ afterwards
# (tools/save_profiles.sh <round>).
set -e
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 300 python bench.py > gpurun_out/bench.jsonl 2> gpurun_out/bench.err
tail -1 gpurun_out/bench.jsonl | cut -c1-400
# the driver's exact form, and rocprof of it (the ramp is in its first launches)
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver_form.jsonl \
  2> gpurun_out/bench_driver_form.err
tail -1 gpurun_out/bench_driver_form.jsonl | cut -c1-300
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_driver_form -o run -- \
  python3 bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/bench_driver_form_prof.jsonl \
  2> gpurun_out/bench_driver_form_prof.err
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- \
  python3 bench.py --cpu-baseline-seconds 0 > gpurun_out/bench_prof.jsonl 2> gpurun_out/bench_prof.err
tail -1 gpurun_out/bench_prof.jsonl | cut -c1-300
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_server -o run -- \
  python3 tools/server_bench.py > gpurun_out/server_bench_prof.jsonl 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- \
  python3 tools/kernel_bench.py --shapes 8:1,8:2,8:4,8:8,32:8 --rounds 1 --reps 2 --calib 8 --bipartite > gpurun_out/pmc_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- \
  python3 tools/kernel_bench.py --shapes 8:1,8:2,8:4,8:8,32:8 --rounds 1 --reps 2 --calib 8 --bipartite > gpurun_out/pmc_write.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_server_fetch -o run -- \
  python3 tools/server_bench.py --reps 3 > gpurun_out/pmc_server_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_server_write -o run -- \
  python3 tools/server_bench.py --reps 3 > gpurun_out/pmc_server_write.log 2>&1
tools/pmc_sq.sh 8:1,8:2,8:4,8:8,32:8 > /dev/null
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dp -o run -- \
  python3 tools/dp_bench.py --reps 10 --passes 1 > gpurun_out/dp_bench_prof.jsonl 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_dp_fetch -o run -- \
  python3 tools/dp_bench.py --reps 2 --passes 1 --warmup 0 > gpurun_out/pmc_dp_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_dp_write -o run -- \
  python3 tools/dp_bench.py --reps 2 --passes 1 --warmup 0 > gpurun_out/pmc_dp_write.log 2>&1
timeout -k 10 200 python tools/dp_bench.py > gpurun_out/dp_bench.jsonl 2>&1
timeout -k 10 120 python -u tools/kernel_bench.py --rounds 5 > gpurun_out/kb_shapes.jsonl
timeout -k 10 120 tools/microbench/draw_ops > gpurun_out/draw_ops.jsonl
timeout -k 10 200 tools/microbench/stream_rate > gpurun_out/stream_rate.jsonl
timeout -k 10 200 python tools/server_bench.py > gpurun_out/server_bench.jsonl 2>&1
timeout -k 10 400 python bench.py --extra --cpu-baseline-seconds 0 > gpurun_out/bench_extra.jsonl 2> gpurun_out/bench_extra.err
timeout -k 10 300 python bench.py --gpus 1 --dist --steps 500 --cpu-baseline-seconds 0 > gpurun_out/bench_dist_world1.jsonl 2> gpurun_out/bench_dist_world1.err
echo PROFILE_OK
