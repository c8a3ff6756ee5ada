set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 200 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_dp -o run -- \
  python3 tools/dp_bench.py --reps 10 --passes 1 > gpurun_out/dp_bench_prof.jsonl 2>&1
timeout -s KILL 120 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_dp_fetch -o run -- \
  python3 tools/dp_bench.py --reps 2 --passes 1 --warmup 0 > gpurun_out/pmc_dp_fetch.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_dp_write -o run -- \
  python3 tools/dp_bench.py --reps 2 --passes 1 --warmup 0 > gpurun_out/pmc_dp_write.log 2>&1
echo DP_PMC_OK
