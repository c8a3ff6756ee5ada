# round 5: the DP norm / clip change and the multi-launch schedule, on the GPU
set -o pipefail
mkdir -p gpurun_out/r05
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread -m gpu \
  tests/test_gpu_dp.py tests/test_gpu_multi_launch.py tests/test_gpu_c_abi.py tests/test_gpu_aggregator.py \
  > gpurun_out/r05/dp_multilaunch_tests.log 2>&1 || exit 1
timeout -k 10 200 python tools/dp_bench.py > gpurun_out/r05/dp_bench.jsonl 2>&1 || exit 1
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/r05/prof_dp -o run -- \
  python3 tools/dp_bench.py --reps 10 --passes 1 > gpurun_out/r05/dp_bench_prof.jsonl 2>&1 || exit 1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/r05/pmc_dp_fetch -o run -- \
  python3 tools/dp_bench.py --reps 2 --passes 1 --warmup 0 > gpurun_out/r05/pmc_dp_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/r05/pmc_dp_write -o run -- \
  python3 tools/dp_bench.py --reps 2 --passes 1 --warmup 0 > gpurun_out/r05/pmc_dp_write.log 2>&1
