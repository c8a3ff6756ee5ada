export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 500 python -m pytest tests -x -q -m gpu > gpurun_out/pytest_gpu.log 2>&1 || { echo "pytest failed"; tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -2 gpurun_out/pytest_gpu.log
timeout -k 10 200 python tools/kernel_bench.py > gpurun_out/kb.json 2>&1 && cat gpurun_out/kb.json &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d gpurun_out/prof_bench -o run -- python bench.py --steps 10 --warmup 2 --cpu-baseline-seconds 0 > gpurun_out/bench_prof.log 2>&1 && tail -1 gpurun_out/bench_prof.log &&
timeout -k 10 300 rocprofv3 --pmc FETCH_SIZE --output-format csv -d gpurun_out/pmc_fetch -o run -- python tools/kernel_bench.py --shapes 8:1 --rounds 1 --reps 2 --calib 8 > gpurun_out/pmc_fetch.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc WRITE_SIZE --output-format csv -d gpurun_out/pmc_write -o run -- python tools/kernel_bench.py --shapes 8:1 --rounds 1 --reps 2 --calib 8 > gpurun_out/pmc_write.log 2>&1 && echo PMC_OK
