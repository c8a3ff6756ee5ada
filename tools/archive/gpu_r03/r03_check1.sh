set -o pipefail
export TMPDIR=/tmp
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_rccl.py "tests/test_gpu_parity.py::test_server_kernels_sizes_and_alignment" "tests/test_gpu_parity.py::test_full_size_properties" > gpurun_out/t1.log 2>&1 || { tail -30 gpurun_out/t1.log; exit 1; }
tail -3 gpurun_out/t1.log
timeout -k 10 200 python tools/server_bench.py > gpurun_out/server_bench.jsonl 2>&1 || { cat gpurun_out/server_bench.jsonl; exit 1; }
cat gpurun_out/server_bench.jsonl
timeout -k 10 300 python bench.py --steps 500 > gpurun_out/bench_quick.jsonl 2> gpurun_out/bench_quick.err || { tail gpurun_out/bench_quick.err; exit 1; }
cut -c1-1500 gpurun_out/bench_quick.jsonl
