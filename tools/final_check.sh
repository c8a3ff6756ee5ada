#!/bin/bash
# Round-end check on one box, in the driver's order: the -m gpu suite,
# smoke(), and bench.py in the driver's N = 1 form.
set -e
mkdir -p gpurun_out/final
timeout -k 10 700 python -u -m pytest -x -v --timeout 200 --timeout-method thread -m gpu tests/ \
  > gpurun_out/final/gpu_suite.log 2>&1
tail -1 gpurun_out/final/gpu_suite.log
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final/smoke.log 2>&1
cat gpurun_out/final/smoke.log
timeout -k 10 300 python bench.py --gpus 1 --steps 20 --warmup 5 > gpurun_out/final/bench_driver_form.jsonl \
  2> gpurun_out/final/bench_driver_form.err
tail -1 gpurun_out/final/bench_driver_form.jsonl | cut -c1-300
