#!/bin/bash
# The server's sum_decode on vectors that are NOT pooled results (fresh
# arrays, as deserialised from the parties' processes): registered lazily
# (SFL_SERVER_REGISTER=1) vs staged through the feeder (0), 8 x 100M,
# interleaved twice; after the pipeline tests.
set -e
mkdir -p gpurun_out/srvreg
timeout -k 10 300 python -u -m pytest -x -v --timeout 120 --timeout-method thread tests/test_gpu_party_pipeline.py \
  > gpurun_out/srvreg/pipeline_tests.log 2>&1
tail -1 gpurun_out/srvreg/pipeline_tests.log
for rep in 1 2; do
  for R in 1 0; do
    SFL_SERVER_REGISTER=$R SFL_HOSTPIPE_TRACE=1 timeout -k 10 240 python tools/party_bench.py --fresh-wires --reps 3 \
      > gpurun_out/srvreg/reg${R}_rep$rep.jsonl 2> gpurun_out/srvreg/reg${R}_rep$rep.trace
  done
done
